"""Which gradients the fused clip norm covers (dW GEMM partials) on a 2-layer Llama-3.1-8B-shaped
model, one step at the config-2 batch (diagnostic for mxllm/train/trainer.py ``_fused_sq``)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from mxllm.models import Llama, get_config  # noqa: E402
from mxllm.parallel.runtime import DistEnv  # noqa: E402
from mxllm import ops  # noqa: E402
from mxllm.train.trainer import OptimConfig, Trainer  # noqa: E402

dev = torch.device("cuda", 0)
cfg = get_config("llama3.1-8b").replace(n_layers=2)
model = Llama(cfg, device=dev, dtype=torch.bfloat16, seed=0)
tr = Trainer(model, DistEnv(device=dev, backend="nccl"), OptimConfig(lr=1e-4))
ids = torch.randint(0, cfg.vocab_size, (2, 2048), device=dev)
import importlib  # noqa: E402

linear = importlib.import_module("mxllm.ops.linear")
from mxllm.ops import gemm  # noqa: E402

_real_mm_sq = gemm.mm_sq


def _traced_mm_sq(form, a, b, out, sq, alpha_t=None):
    ok = _real_mm_sq(form, a, b, out, sq, alpha_t)
    M, N, K = gemm._dims(form, a, b)
    print(f"mm_sq {form} M{M} N{N} K{K} a{tuple(a.shape)}/{a.stride()} {a.dtype} b{tuple(b.shape)}/{b.stride()} "
          f"out{out.dtype} sched={gemm.schedule(form, M, N, K, torch.bfloat16)} -> {ok}")
    return ok


gemm.mm_sq = _traced_mm_sq
_real_pwg = linear.param_weight_grad


def _traced_pwg(wp, dy, x, dy_scale=None):
    if wp is not None and getattr(wp, "_mx_sq", None) is not None:
        print(f"param_weight_grad {tuple(wp.shape)} fresh={getattr(wp, '_mx_grad_fresh', None)} "
              f"armed={getattr(wp, '_mx_sq_done', None)} dy{dy.dtype} x{x.dtype}")
    return _real_pwg(wp, dy, x, dy_scale)


linear.param_weight_grad = _traced_pwg
_fused = importlib.import_module("mxllm.ops.fused")
_loss = importlib.import_module("mxllm.ops.loss")

_fused.param_weight_grad = _traced_pwg
_loss.param_weight_grad = _traced_pwg
for _ in range(2):
    tr.train_step([(ids, ids)])
    torch.cuda.synchronize()
    # the full pass over the same (still present: overwrite-style) gradient, for comparison
    full = float(ops.sq_norm(tr.flat.grads).sqrt())
    print(f"clip norm fused {float(tr.last_grad_norm):.8g} full pass {full:.8g} "
          f"rel diff {abs(float(tr.last_grad_norm) - full) / full:.3g}")
torch.cuda.synchronize()
names = {id(p): n for n, p in model.named_parameters()}
for p in tr._sq_params:
    print(f"{names[id(p)]:40s} {tuple(p.shape)} done={p._mx_sq_done}")
big, small = next(iter(tr._sq_plan.values())) if tr._sq_plan else ([], [])
print("plans", len(tr._sq_plan), "big ranges", len(big), "small ranges", len(small))
