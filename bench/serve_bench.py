#!/usr/bin/env python3
"""Inference-engine benchmark (the local replacement of the reference's remote
Llama-3.1-70B completion endpoint, reference src/distributed_inference.py:34-41).

Measures on one GPU, random-init bf16 weights, synthetic prompts:
  * prefill: tokens/s and TTFT for one prompt of --prompt-len tokens;
  * decode: ms/step and tokens/s of the hipGraph-replayed decode step at each
    batch size in --batches (context --ctx tokens per sequence), with the
    achieved weight-streaming bandwidth (bf16 weight bytes / step time: decode
    at small batch is bound by reading every weight once per step);
  * end-to-end: Engine.generate over --requests prompts (continuous batching),
    output tokens/s and mean TTFT.
Prints one JSON line (and writes it to --json-out).

Tensor parallelism (mxllm/parallel/tensor.py):
  * ``torchrun --nproc-per-node=N bench/serve_bench.py --model llama3.1-70b``:
    every rank serves its TP shard, two RCCL all-reduces per layer and a
    vocab-parallel head inside the graphed decode step; rank 0 reports;
  * ``--tp-shard-proxy N`` (one GPU): rank 0's shard of a TP-N deployment with
    the collectives left out — the per-GPU compute floor of a TP-N decode step.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3.1-8b")
    ap.add_argument("--prompt-len", type=int, default=1024)
    ap.add_argument("--ctx", type=int, default=1024, help="cached tokens per sequence in the decode sweep")
    ap.add_argument("--batches", default="1,8,32,64")
    ap.add_argument("--decode-steps", type=int, default=32)
    ap.add_argument("--requests", type=int, default=64)
    ap.add_argument("--new-tokens", type=int, default=64)
    ap.add_argument("--e2e-prompt-len", type=int, default=256)
    ap.add_argument("--fp8", action="store_true", help="e4m3 projection weights (serving quantisation)")
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--top-p", type=float, default=1.0, help="e2e requests: nucleus sampling (with --temperature)")
    ap.add_argument("--temperature", type=float, default=0.0)
    ap.add_argument("--kv-pool-tokens", type=int, default=None,
                    help="paged KV cache shared by all slots (default: every slot owns max_seq positions)")
    ap.add_argument("--tp-shard-proxy", type=int, default=0,
                    help="one GPU: run rank 0's TP-N shard without the collectives (per-GPU compute floor)")
    a = ap.parse_args()

    from mxllm.models import Llama, get_config
    from mxllm.serve.engine import Engine
    from mxllm.utils import gemm_tuning

    gemm_tuning.enable()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    tp_group, rank = None, 0
    if world > 1:
        import torch.distributed as dist

        from mxllm.parallel import runtime

        env = runtime.init()
        dev, rank, tp_group = env.device, env.rank, dist.group.WORLD
    else:
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
    cfg = get_config(a.model)
    t0 = time.perf_counter()
    tp = world if world > 1 else a.tp_shard_proxy
    if tp > 1:
        from mxllm.parallel.tensor import random_shard

        model = random_shard(cfg, rank, tp, dev, seed=0)
    else:
        model = Llama(cfg, device=dev, dtype=torch.bfloat16, seed=0)
    model.requires_grad_(False)
    full_cfg, cfg = cfg, model.cfg  # per-rank shapes from here on (KV bytes, prompts use the vocab below)
    if a.fp8:
        from mxllm.serve.quant import quantize_model_fp8_

        quantize_model_fp8_(model)
    torch.cuda.synchronize()
    init_s = time.perf_counter() - t0
    wbytes = sum(p.numel() * p.element_size() for p in model.parameters()) + \
        sum(b.numel() * b.element_size() for n, b in model.named_buffers() if n.endswith((".q", ".scale")))
    bmax = max(int(b) for b in a.batches.split(","))
    max_seq = max(a.prompt_len, a.ctx + a.decode_steps, a.e2e_prompt_len + a.new_tokens) + 8
    eng = Engine(model, max_batch=max(bmax, 1), max_seq=max_seq, tp_group=tp_group, kv_pool_tokens=a.kv_pool_tokens)
    g = torch.Generator().manual_seed(0)

    def prompt(n):
        return torch.randint(0, full_cfg.vocab_size, (n,), generator=g).tolist()

    # ---- prefill / TTFT
    eng.prefill(0, prompt(a.prompt_len))  # warm-up (library handles)
    torch.cuda.synchronize()
    times = []
    for _ in range(3):
        t = time.perf_counter()
        logits = eng.prefill(0, prompt(a.prompt_len))
        nxt = int(logits.argmax())  # TTFT includes the first token's read-back
        times.append(time.perf_counter() - t)
    del nxt
    pre_s = min(times)
    out = {"model": a.model, "weights": "fp8-e4m3 projections" if a.fp8 else "bf16",
           "tensor_parallel": ({"tp": world, "collectives": "RCCL all-reduce x2/layer + logits all-gather"}
                               if world > 1 else
                               {"tp": a.tp_shard_proxy, "collectives": "omitted (one-GPU shard proxy)"}
                               if a.tp_shard_proxy > 1 else None),
           "weights_gb": round(wbytes / 1e9, 1), "init_s": round(init_s, 1),
           "prefill": {"prompt_len": a.prompt_len, "ttft_ms": round(1e3 * pre_s, 2),
                       "tokens_per_s": round(a.prompt_len / pre_s, 1)},
           "decode": []}

    # ---- decode sweep (graphed step; every sequence holds --ctx cached tokens)
    for bs in [int(b) for b in a.batches.split(",")]:
        slots = list(range(bs))
        for s in slots:
            eng.reserve(s, a.ctx + 4 * a.decode_steps + 8)  # paged KV: this slot's blocks (static: no-op)
            eng.lens[s] = a.ctx
        tok = torch.randint(0, full_cfg.vocab_size, (bs,), generator=g)
        for _ in range(3):  # capture + warm
            eng.decode(slots, tok)
        for s in slots:
            eng.lens[s] = a.ctx
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(a.decode_steps):
            eng.decode(slots, tok)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / a.decode_steps
        kv_bytes = bs * (a.ctx + a.decode_steps // 2) * cfg.n_layers * 2 * cfg.n_kv_heads * cfg.head_dim * 2
        out["decode"].append({"batch": bs, "ctx": a.ctx, "ms_per_step": round(1e3 * dt, 3),
                              "tokens_per_s": round(bs / dt, 1),
                              "weight_stream_tb_s": round(wbytes / dt / 1e12, 2),
                              "hbm_tb_s_weights_plus_kv": round((wbytes + kv_bytes) / dt / 1e12, 2)})
        if bs == bmax:  # decode step + batched sampling + token read-back: greedy vs T 0.8 / top-p 0.9
            from mxllm.ops import decode as dops

            for mode, (tt, tp_) in (("greedy", (0.0, 1.0)), ("t0.8_top_p0.9", (0.8, 0.9))):
                for s in slots:
                    eng.lens[s] = a.ctx
                torch.cuda.synchronize()
                t = time.perf_counter()
                for i in range(a.decode_steps):
                    lg = eng.decode(slots, tok)
                    dops.sample_rows(lg[:bs], [tt] * bs, [tp_] * bs, [0] * bs, list(range(bs)), [i] * bs).tolist()
                dt2 = (time.perf_counter() - t) / a.decode_steps
                out.setdefault("decode_plus_sampling", {})[mode] = {"batch": bs, "ms_per_step": round(1e3 * dt2, 3)}
        for s in slots:
            eng.lens[s] = 0
            eng.kv.release(s)

    # ---- end-to-end continuous batching
    if a.requests > 0:
        eng2 = eng
        prompts = [prompt(a.e2e_prompt_len) for _ in range(a.requests)]
        eng2.generate(prompts[:2], max_new_tokens=4)  # warm
        f0, ttft0, n0 = eng2.finished, eng2.ttft_sum, eng2.tokens_generated
        torch.cuda.synchronize()
        t = time.perf_counter()
        outs = eng2.generate(prompts, max_new_tokens=a.new_tokens, temperature=a.temperature, top_p=a.top_p)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
        ntok = sum(len(o) for o in outs)
        out["e2e"] = {"requests": a.requests, "prompt_len": a.e2e_prompt_len, "new_tokens": a.new_tokens,
                      "temperature": a.temperature, "top_p": a.top_p,
                      "max_batch": eng2.max_batch, "wall_s": round(dt, 3),
                      "output_tokens_per_s": round(ntok / dt, 1),
                      "total_tokens_per_s": round((ntok + a.requests * a.e2e_prompt_len) / dt, 1),
                      "mean_ttft_ms": round(1e3 * (eng2.ttft_sum - ttft0) / max(1, eng2.finished - f0), 1),
                      "kv_cache": ({"paged": True, "pool_tokens": a.kv_pool_tokens, "block": eng2.kv.block,
                                    "gb": round(eng2.kv.nbytes() / 1e9, 2)} if eng2.kv.paged else
                                   {"paged": False, "gb": round(eng2.kv.nbytes() / 1e9, 2)})}
    if rank == 0:
        line = json.dumps(out)
        print(line, flush=True)
        if a.json_out:
            with open(a.json_out, "w") as f:
                f.write(line + "\n")
    if world > 1:
        runtime.cleanup()


if __name__ == "__main__":
    main()
