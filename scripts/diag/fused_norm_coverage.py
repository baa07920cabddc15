"""Which gradients the fused clip norm covers (dW GEMM partials) on a 2-layer Llama-3.1-8B-shaped
model, one step at the config-2 batch (diagnostic for mxllm/train/trainer.py ``_fused_sq``)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from mxllm.models import Llama, get_config  # noqa: E402
from mxllm.parallel.runtime import DistEnv  # noqa: E402
from mxllm.train.trainer import OptimConfig, Trainer  # noqa: E402

dev = torch.device("cuda", 0)
cfg = get_config("llama3.1-8b").replace(n_layers=2)
model = Llama(cfg, device=dev, dtype=torch.bfloat16, seed=0)
tr = Trainer(model, DistEnv(device=dev, backend="nccl"), OptimConfig(lr=1e-4))
ids = torch.randint(0, cfg.vocab_size, (2, 2048), device=dev)
for _ in range(2):
    tr.train_step([(ids, ids)])
torch.cuda.synchronize()
names = {id(p): n for n, p in model.named_parameters()}
for p in tr._sq_params:
    print(f"{names[id(p)]:40s} {tuple(p.shape)} done={p._mx_sq_done}")
big, small = next(iter(tr._sq_plan.values())) if tr._sq_plan else ([], [])
print("plans", len(tr._sq_plan), "big ranges", len(big), "small ranges", len(small))
