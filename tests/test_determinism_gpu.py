"""Deterministic training mode (reference docs/troubleshooting.md:60-62).

``MXLLM_DETERMINISTIC=1`` routes every GEMM of the step that the 8-phase MFMA kernel takes
(csrc/kernels/gemm8.hip: one workgroup per output tile, a fixed K order, no split-K, no atomics)
through it instead of hipBLASLt / rocBLAS, whose stream-K / atomic solutions made two identical
runs diverge (archive/profiles/r3aa).  Every other kernel of the step is already fixed-order (attention's
default split backward, sorted embedding backward, fixed-order norms / CE / grad norm, elementwise
AdamW).  Two from-scratch Llama-3.2-1B full fine-tunes must then agree bitwise: every step's loss
and every final weight.
"""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(gpu, steps: int):
    from mxllm.data import SyntheticTokens
    from mxllm.models import Llama, get_config
    from mxllm.parallel.runtime import DistEnv
    from mxllm.train.trainer import OptimConfig, Trainer

    cfg = get_config("llama3.2-1b")
    torch.manual_seed(0)
    model = Llama(cfg, device=gpu, dtype=torch.bfloat16, seed=1234)
    tr = Trainer(model, DistEnv(device=gpu, backend="nccl"), OptimConfig(lr=1e-4, weight_decay=0.01, grad_clip=1.0))
    data = SyntheticTokens(cfg.vocab_size, 8, 512, gpu, seed=1)
    batches = [data.next() for _ in range(4)]  # cycled: random tokens are only learnable by repetition
    losses = [tr.train_step([batches[i % 4]]) for i in range(steps)]
    torch.cuda.synchronize()
    tr.params_ready()
    out = ([float(x) for x in losses], tr.master_fp32().clone())
    del tr, model
    torch.cuda.empty_cache()
    return out


def test_deterministic_mode_two_runs_bitwise(gpu, monkeypatch):
    from mxllm.ops import gemm

    monkeypatch.setenv("MXLLM_DETERMINISTIC", "1")
    assert gemm.deterministic()
    # every projection / head GEMM of this config is a shape the kernel takes
    for form, M, N, K in (("tn", 4096, 3072, 2048), ("nn", 4096, 2048, 3072), ("tt", 3072, 2048, 4096),
                          ("tn", 4096, 128256, 2048), ("nn", 4096, 2048, 128256), ("tt", 128256, 2048, 4096)):
        assert gemm.want(form, M, N, K, torch.bfloat16)
    l1, w1 = _run(gpu, 100)
    l2, w2 = _run(gpu, 100)
    assert l1[-1] < l1[0]  # it trains
    first = next((i for i, (a, b) in enumerate(zip(l1, l2)) if a != b), None)
    assert first is None, f"losses differ from step {first}: {l1[first]} vs {l2[first]}"
    assert torch.equal(w1, w2)
