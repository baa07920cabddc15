"""Why do the fused-clip-norm and full-pass trainers leave the same trajectory?  Runs the
tests/test_train_gpu.py::test_fused_grad_norm_matches_full_pass setup (tiny-d128, 3 layers, MXLLM_GEMM8=all)
three times -- fused, full pass, full pass again -- and prints, per step, each parameter's gradient max-abs
difference against the first full-pass run (bitwise equal gradients print 0), plus the norms."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
os.environ["MXLLM_GEMM8"] = "all"

from mxllm.models import Llama, get_config  # noqa: E402
from mxllm.parallel.runtime import DistEnv  # noqa: E402
from mxllm.parallel.zero3 import init_full_state  # noqa: E402
from mxllm.train.trainer import OptimConfig, Trainer  # noqa: E402


def run(fused):
    os.environ["MXLLM_FUSED_GRAD_NORM"] = fused
    gpu = torch.device("cuda:0")
    cfg = get_config("tiny-d128").replace(n_layers=3, vocab_size=1024)
    model = Llama(cfg, device=gpu, seed=0)
    sd = init_full_state(cfg, 5, gpu)
    with torch.no_grad():
        for n, p in model.named_parameters():
            p.copy_(sd[n])
    tr = Trainer(model, DistEnv(device=gpu, backend="nccl"), OptimConfig(lr=1e-3, weight_decay=0.01))
    g = torch.Generator(device=gpu).manual_seed(3)
    batches = [torch.randint(0, cfg.vocab_size, (2, 256), device=gpu, generator=g) for _ in range(3)]
    steps = []
    for b in batches:
        tr.train_step([(b, b)])
        torch.cuda.synchronize()
        grads = {s.name: tr.flat.grads[s.offset:s.offset + s.numel].float().clone() for s in tr.flat.slots}
        steps.append((float(tr.last_grad_norm), grads))
    return steps


def main():
    print("cfg heads / head_dim:", get_config("tiny-d128").n_heads, get_config("tiny-d128").head_dim)
    ref = run("0")
    for label, fused in (("full-pass again", "0"), ("fused", "1")):
        other = run(fused)
        print(f"== {label} vs full pass")
        for i, ((n0, g0), (n1, g1)) in enumerate(zip(ref, other)):
            print(f"step {i}: norm {n0:.9g} vs {n1:.9g}")
            for k in g0:
                d = (g0[k] - g1[k]).abs().max().item()
                if d:
                    print(f"   {k}: max|dg| {d:.3e} (max|g| {g0[k].abs().max().item():.3e})")


if __name__ == "__main__":
    main()
