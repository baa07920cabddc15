"""Tune hipBLASLt/rocBLAS solutions (PyTorch TunableOp) for the DECODE GEMMs of
the serving engine — y = x W^T with 1..64 token rows (the engine's power-of-two
decode buckets) for every projection and the LM head — and merge them into the
selection table used read-only at run time (mxllm/utils/gemm_tuning.py).

Decode GEMMs stream the weights from HBM once per step, so the tuning runs with
a rotating operand buffer larger than the 256 MB Infinity Cache: a solution is
picked for cold weights, not for operands left in cache by the previous timing
iteration.  The engine runs eager here (MXLLM_DECODE_GRAPHS=0) so every GEMM is
a plain library call TunableOp sees; the graphed engine replays the same
solutions.  Prints the default and tuned per-step decode time per bucket.

  python bench/tune_decode_gemms.py --model llama3.1-8b --out gpurun_out/tune_decode.csv [--prefill 1024]
"""
import argparse
import json
import os
import sys
import time

os.environ.setdefault("MXLLM_DECODE_GRAPHS", "0")
import torch  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def step_ms(eng, bs, ctx, vocab, steps=8):
    slots = list(range(bs))
    tok = torch.randint(0, vocab, (bs,))
    for s in slots:
        eng.lens[s] = ctx
    eng.decode(slots, tok)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(steps):
        eng.decode(slots, tok)
    torch.cuda.synchronize()
    return 1e3 * (time.perf_counter() - t) / steps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3.1-8b")
    ap.add_argument("--batches", default="1,2,4,8,16,32,64")
    ap.add_argument("--ctx", type=int, default=512)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "tune_decode.csv"))
    ap.add_argument("--max-ms", type=int, default=30, help="TunableOp time budget per candidate solution")
    ap.add_argument("--rotating-mb", type=int, default=512)
    ap.add_argument("--prefill", default="", help="also tune the prefill GEMMs of these prompt lengths (e.g. 1024)")
    a = ap.parse_args()

    from mxllm.models import Llama, get_config
    from mxllm.serve.engine import Engine
    from mxllm.utils import gemm_tuning

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    cfg = get_config(a.model)
    model = Llama(cfg, device=dev, dtype=torch.bfloat16, seed=0)
    model.requires_grad_(False)
    batches = [int(b) for b in a.batches.split(",")]
    plens = [int(x) for x in a.prefill.split(",") if x]
    eng = Engine(model, max_batch=max(batches), max_seq=max([a.ctx + 64] + [n + 8 for n in plens]))
    res = {"model": a.model, "ctx": a.ctx, "default_ms": {}, "tuned_ms": {}}

    def prefill_ms(n, reps=3):
        ids = torch.randint(0, cfg.vocab_size, (n,)).tolist()
        eng.prefill(0, ids)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(reps):
            eng.prefill(0, ids)
        torch.cuda.synchronize()
        return 1e3 * (time.perf_counter() - t) / reps
    gemm_tuning.enable()  # the current table: training shapes; decode shapes fall back to the library default
    for bs in batches:
        res["default_ms"][bs] = round(step_ms(eng, bs, a.ctx, cfg.vocab_size), 3)
    for n in plens:
        res["default_ms"][f"prefill{n}"] = round(prefill_ms(n), 3)
    print(json.dumps({"phase": "default", **res["default_ms"]}), flush=True)

    tun = torch.cuda.tunable
    tun.set_filename(a.out, insert_device_ordinal=False)
    tun.set_rotating_buffer_size(a.rotating_mb)
    tun.set_max_tuning_duration(a.max_ms)
    tun.tuning_enable(True)
    t0 = time.time()
    for bs in batches:
        step_ms(eng, bs, a.ctx, cfg.vocab_size, steps=1)
        print(json.dumps({"phase": "tuning", "batch": bs, "elapsed_s": round(time.time() - t0, 1)}), flush=True)
    for n in plens:
        prefill_ms(n, reps=1)
        print(json.dumps({"phase": "tuning", "prefill": n, "elapsed_s": round(time.time() - t0, 1)}), flush=True)
    tun.tuning_enable(False)  # the results stay in memory; TunableOp writes a.out at process exit
    for bs in batches:
        res["tuned_ms"][bs] = round(step_ms(eng, bs, a.ctx, cfg.vocab_size), 3)
    for n in plens:
        res["tuned_ms"][f"prefill{n}"] = round(prefill_ms(n), 3)
    print(json.dumps({"phase": "tuned", **res["tuned_ms"]}), flush=True)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
