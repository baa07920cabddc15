"""A/B of the two lora_xwt kernels (csrc/kernels/lora.hip) at the Llama-3.1-70B
LoRA shapes (T = 4096 tokens, pad 64): the register-fragment kernel
(MXLLM_LORA_XWT=reg) vs the LDS-DMA-staged one (default), the latter also with its
split reduction merged in-launch (MXLLM_LORA_FUSED_RED=1, "lds_f"), interleaved rounds
in ONE process; prints the median us/call and the streamed operand's bandwidth."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

T, r, P = 4096, 16, 64
PROJ = {"qkv": (8192, 10240), "o": (8192, 8192), "gu": (8192, 57344), "down": (28672, 8192)}


def timeit(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return 1e3 * a.elapsed_time(b) / iters


def setv(v):
    os.environ["MXLLM_LORA_XWT"] = "reg" if v == "reg" else "lds"
    os.environ["MXLLM_LORA_FUSED_RED"] = "1" if v == "lds_f" else "0"


def main():
    from mxllm.ops import _ext

    nat = _ext.native()
    res = []
    tot = {"reg": 0.0, "lds": 0.0, "lds_f": 0.0}
    for name, (K, N) in PROJ.items():
        wbuf = torch.randn(N + P, K + P, device="cuda", dtype=torch.bfloat16) * 0.02
        xa = torch.randn(T, K + P, device="cuda", dtype=torch.bfloat16)
        dya = torch.randn(T, N + P, device="cuda", dtype=torch.bfloat16)
        bt = wbuf[:N, K:].t().contiguous()
        calls = {"fwd": (lambda: nat.lora_xwt(xa[:, :K], wbuf[N:, :K], xa[:, K:], 2.0), T * K * 2),
                 "bwd": (lambda: nat.lora_xwt(dya[:, :N], bt, dya[:, N:], 2.0), T * N * 2)}
        for cname, (fn, nbytes) in calls.items():
            # numerics: both kernels vs fp32
            outs = {}
            for v in ("reg", "lds", "lds_f"):
                setv(v)
                fn()
                torch.cuda.synchronize()
                outs[v] = (xa[:, K:] if cname == "fwd" else dya[:, N:]).float().clone()
            diff = (outs["reg"] - outs["lds"]).abs().max().item()
            same = bool(torch.equal(outs["lds"], outs["lds_f"]))
            t = {"reg": [], "lds": [], "lds_f": []}
            for _ in range(7):
                for v in ("reg", "lds", "lds_f"):
                    setv(v)
                    t[v].append(timeit(fn))
            med = {v: statistics.median(x) for v, x in t.items()}
            for v in med:
                tot[v] += med[v]
            row = {"proj": name, "call": cname, "MB": round(nbytes / 1e6, 1), "max_abs_diff": diff, "fused_red_bitwise": same}
            for v in med:
                row[f"{v}_us"] = round(med[v], 1)
                row[f"{v}_TBps"] = round(nbytes / med[v] / 1e6, 2)
            print(json.dumps(row), flush=True)
            res.append(row)
        del wbuf, xa, dya, bt
    os.environ.pop("MXLLM_LORA_XWT", None)
    os.environ.pop("MXLLM_LORA_FUSED_RED", None)
    print(json.dumps({"layer_us": {k: round(v, 1) for k, v in tot.items()},
                      "step_ms_80_layers": {k: round(v * 80 / 1e3, 2) for k, v in tot.items()}}), flush=True)


if __name__ == "__main__":
    main()
