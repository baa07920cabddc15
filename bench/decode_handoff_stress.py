"""Correctness stress + timing of the in-launch split-K merge protocols of the decode
attention (csrc/kernels/decode.hip, MXLLM_DECODE_HANDOFF 1..4) against the two-launch
form (combine kernel).  Every protocol runs 300 calls per shape; any output that differs
bitwise from the combine-kernel output is counted.  Also times each form (us per call)."""
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from mxllm.ops import native

    nat = native()
    dev = "cuda"
    torch.manual_seed(0)
    shapes = [("rep4", 128, 8, 2, [0, 5, 63, 255, 256, 300, 640], 700),
              ("rep16", 128, 16, 1, [0, 5, 63, 255, 256, 300, 640], 700),
              ("8b_b1", 128, 32, 8, [1023], 1024),
              ("8b_b64", 128, 32, 8, [1023 - (i % 7) for i in range(64)], 1024)]
    for name, D, Hq, Hkv, lens, max_seq in shapes:
        B = len(lens)
        kc = torch.randn(B, Hkv, max_seq, D, device=dev, dtype=torch.bfloat16)
        vc = torch.randn_like(kc)
        q = torch.randn(B, Hq, D, device=dev, dtype=torch.bfloat16)
        pos = torch.tensor(lens, dtype=torch.int32, device=dev)
        slots = torch.arange(B, dtype=torch.int32, device=dev)
        ml = max(lens) + 1
        sc = 1.0 / math.sqrt(D)
        os.environ["MXLLM_DECODE_HANDOFF"] = "0"
        ref = nat.decode_attn(q, kc, vc, pos, slots, ml, sc, 1)
        cnt = torch.zeros(B * Hkv, dtype=torch.int32, device=dev)
        row = {"shape": name, "B": B, "Hq": Hq, "Hkv": Hkv}
        for proto in (0, 1, 2, 3, 4):
            os.environ["MXLLM_DECODE_HANDOFF"] = str(proto)
            bad = 0
            for _ in range(300):
                o = nat.decode_attn(q, kc, vc, pos, slots, ml, sc, 1, None, cnt)
                bad += int(not torch.equal(o, ref))
            torch.cuda.synchronize()
            a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(100):
                nat.decode_attn(q, kc, vc, pos, slots, ml, sc, 1, None, cnt)
            e.record()
            torch.cuda.synchronize()
            row[f"p{proto}_bad"] = bad
            row[f"p{proto}_us"] = round(a.elapsed_time(e) * 10, 2)
            row[f"p{proto}_cnt_zero"] = int(cnt.abs().sum()) == 0
        print(json.dumps(row), flush=True)
    os.environ.pop("MXLLM_DECODE_HANDOFF", None)


if __name__ == "__main__":
    main()
