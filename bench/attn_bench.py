"""Attention kernel microbenchmark at the Llama-3.1-70B training shape
(B=2, Hq=64, Hkv=8, S=2048, D=128, causal), random data.  Prints TFLOP/s
(causal FLOPs: fwd 2*2*B*Hq*S^2*D/2, bwd 2.5x fwd)."""
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mxllm.ops import native  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


def main():
    B, Hq, Hkv, S, D = [int(x) for x in (sys.argv[1:6] if len(sys.argv) > 5 else (2, 64, 8, 2048, 128))]
    ops = native()
    dev = "cuda"
    q = torch.randn(B, Hq, S, D, device=dev, dtype=torch.bfloat16)
    k = torch.randn(B, Hkv, S, D, device=dev, dtype=torch.bfloat16)
    v = torch.randn(B, Hkv, S, D, device=dev, dtype=torch.bfloat16)
    sc = 1 / math.sqrt(D)
    o, lse = ops.attn_fwd(q, k, v, True, sc)
    do = torch.randn_like(o)
    fl = 2 * 2 * B * Hq * S * S * D / 2
    res = {"shape": [B, Hq, Hkv, S, D]}
    res["fwd_ms"] = timeit(lambda: ops.attn_fwd(q, k, v, True, sc))
    res["bwd_ms"] = timeit(lambda: ops.attn_bwd(do, q, k, v, o, lse, True, sc))  # default (split) mode
    lite = len(sys.argv) > 6 and sys.argv[6] == "lite"  # long S: default modes only (mode 2's workspace ~ S^2)
    if not lite:
        res["bwd_atomic_ms"] = timeit(lambda: ops.attn_bwd(do, q, k, v, o, lse, True, sc, 1))
        res["bwd_partials_ms"] = timeit(lambda: ops.attn_bwd(do, q, k, v, o, lse, True, sc, 2))
        res["bwd_noatomic_ms"] = timeit(lambda: ops.attn_bwd_ablate(do, q, k, v, o, lse, -1, sc))
        res["bwd_noatomic_TF"] = 2.5 * fl / res["bwd_noatomic_ms"] / 1e9
    cs = torch.rand(S, D // 2, device=dev)
    res["bwd_rope_ms"] = timeit(lambda: ops.attn_bwd_rope(do, q, k, v, o, lse, True, sc, cs, cs, 0))  # into d(qkv)
    res["fwd_TF"] = fl / res["fwd_ms"] / 1e9
    res["bwd_TF"] = 2.5 * fl / res["bwd_ms"] / 1e9
    qkv = torch.randn(B * S, (Hq + 2 * Hkv) * D, device=dev, dtype=torch.bfloat16)
    cos = torch.randn(S, D // 2, device=dev)
    res["rope_split_ms"] = timeit(lambda: ops.rope_split(qkv, cos, cos, B, S, Hq, Hkv, D, None))
    dq, dkp, dvp = ops.attn_bwd(do, q, k, v, o, lse, True, sc)
    res["rope_merge_ms"] = timeit(lambda: ops.rope_merge_bwd(dq, dkp, dvp, cos, cos, B, S, Hq, Hkv, D))
    print(json.dumps({k2: (round(v2, 4) if isinstance(v2, float) else v2) for k2, v2 in res.items()}), flush=True)


if __name__ == "__main__":
    main()
