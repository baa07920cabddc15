#!/usr/bin/env python3
"""The reference's own program, timed: ``src/distributed_inference.py`` main()
(reference src/distributed_inference.py:43-81) on this rank's GPU with the
local engine — IMDB-like 1% train split (250 rows, offline synthetic when the
HF cache is absent), DistributedSampler, batch 4, 3 epochs, one batched
generation per DataLoader batch.  The reference makes one serial remote API
call per prompt (375 per rank at world 2).

Prints one JSON line: wall time of main(), prompts/s, prompt and generated
tokens/s (from the engine's counters), mean TTFT.  Run under torchrun for
world > 1.  Model / epochs / new tokens come from the usual MXLLM_* env vars
(MXLLM_ENGINE_MODEL, MXLLM_EPOCHS, MXLLM_MAX_NEW_TOKENS, ...).
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "src"))


def main():
    import distributed_inference as di  # the reference-compatible driver (src/)
    from mxllm.serve import client

    t0 = time.perf_counter()
    di.main()
    wall = time.perf_counter() - t0
    run = di.RUN
    world = int(os.environ.get("WORLD_SIZE", 1))
    rank = int(os.environ.get("RANK", 0))
    entry = client._LOCAL.get(di.CONFIG["MODEL_NAME"])
    eng = entry[0] if isinstance(entry, tuple) else getattr(entry, "engine", entry)
    st = eng.stats() if hasattr(eng, "stats") else {}
    prompts = -(-run.n_rows // world) * run.epochs
    out = {"workload": "reference src/distributed_inference.py main()", "rank": rank, "world": world,
           "engine_model": eng.cfg.name if hasattr(eng, "cfg") else None,
           "prompts_this_rank": prompts, "batch_size": run.batch_size, "epochs": run.epochs,
           "max_new_tokens": run.max_new_tokens, "wall_s": round(wall, 2),
           "prompts_per_s": round(prompts / wall, 2),
           "prompt_tokens": getattr(eng, "prefill_tokens", None), "generated_tokens": st.get("tokens_generated"),
           "prefill_tokens_per_s": round(st.get("prefill_tokens_per_s", 0.0), 1),
           "decode_tokens_per_s": round(st.get("decode_tokens_per_s", 0.0), 1),
           "mean_ttft_ms": round(1e3 * st.get("mean_ttft_s", 0.0), 1)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
