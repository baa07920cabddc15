"""Same-process A/B of env-switched variants of a bench workload (default: the 8B full fine-tune
step, BASELINE config 2; ``--model llama3.1-70b --finetune lora``: the headline).

Every variant runs ``bench.run`` in THIS process (one model init per variant, rounds
interleaved so clock/thermal drift hits every variant alike) and prints one JSON line:
  {"variant": ..., "round": r, "ms_per_step": ..., "value": ...}
Variants are ``name=ENV1=V1,ENV2=V2`` arguments (env switches read at Trainer init:
MXLLM_ADAMW_CUS, MXLLM_ADAMW_LAG, MXLLM_OVERLAP_ADAMW, ...).

  python bench/adamw_overlap_ab.py --rounds 2 base= cu16=MXLLM_ADAMW_CUS=mod8:1
"""
from __future__ import annotations

import argparse
import gc
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--model", default="llama3.1-8b")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--finetune", default="full", choices=["full", "lora"])
    ap.add_argument("--json-out", default=None)
    ap.add_argument("variants", nargs="+")
    a = ap.parse_args()
    import torch

    import bench
    from mxllm.parallel import runtime

    env = runtime.init()
    variants = []
    for v in a.variants:
        name, _, spec = v.partition("=")
        kv = dict(x.split("=", 1) for x in spec.split(",") if x)
        variants.append((name, kv))
    keys = sorted({k for _, kv in variants for k in kv})
    out = open(a.json_out, "a") if a.json_out else None
    for r in range(a.rounds):
        for name, kv in variants:
            for k in keys:
                os.environ.pop(k, None)
            os.environ.update(kv)
            b = bench.parse(["--model", a.model, "--finetune", a.finetune, "--steps", str(a.steps), "--warmup",
                             str(a.warmup)])
            t0 = time.time()
            try:
                res = bench.run(b, env)
                rec = {"variant": name, "env": kv, "round": r, "ms_per_step": res["ms_per_step"],
                       "value": res["value"], "final_loss": res["final_loss"], "peak_hbm_gb": res["peak_hbm_gb"],
                       "wall_s": round(time.time() - t0, 1)}
            except Exception as e:  # noqa: BLE001
                rec = {"variant": name, "env": kv, "round": r, "error": f"{type(e).__name__}: {e}"[:300]}
            line = json.dumps(rec)
            print(line, flush=True)
            if out:
                out.write(line + "\n")
                out.flush()
            gc.collect()
            torch.cuda.synchronize()
            torch.cuda.empty_cache()
    runtime.cleanup()


if __name__ == "__main__":
    main()
