"""Typed run configuration with precedence CLI > env > CONFIG dict > defaults.

The reference reads a gitignored ``config.CONFIG`` dict (keys MASTER_ADDR,
MASTER_PORT, MODEL_NAME, API_KEY, API_BASE — reference
src/distributed_inference.py:12,15-16,37,53-54) and hard-codes everything else
(dataset/split :56, batch 4 :59, epochs 3 :61, truncation 100 :73-74, backend
"nccl" :17).  Every one of those is a field here with the reference's default;
a CONFIG dict still works (upper-case keys), env vars ``MXLLM_<FIELD>``
override it, CLI flags override env.  torchrun-provided MASTER_ADDR/PORT always
win over CONFIG.
"""
from __future__ import annotations

import argparse
import dataclasses
import os
from dataclasses import dataclass, fields


@dataclass
class RunConfig:
    # reference CONFIG keys
    master_addr: str = "127.0.0.1"
    master_port: int = 29500
    model_name: str = "mxllm/llama3.1-70b"
    api_key: str = ""
    api_base: str = "local"
    # reference hard-coded constants
    dataset: str = "imdb"
    split: str = "train[:1%]"
    n_rows: int = 250
    batch_size: int = 4
    epochs: int = 3
    truncate: int = 100
    backend: str = ""  # "" = auto: nccl (RCCL) with GPUs, gloo on CPU
    seed: int = 0
    # local inference engine
    engine_model: str = ""  # "" = preset from MODEL_NAME on GPU (tiny stub on CPU)
    engine_weights: str = "bf16"  # bf16 | fp8 (e4m3 projection weights for serving, mxllm/serve/quant.py)
    max_new_tokens: int = 32
    temperature: float = 0.0
    max_batch: int = 32
    # inference driver: DataLoader batches kept in flight on the local engine (their
    # prompts are generated together by continuous batching; results are still
    # logged batch by batch, in order).  0 = one batch at a time, as the reference.
    lookahead_batches: int = 8
    # engine context window: long enough for whole IMDB-like reviews (~8k byte tokens at the tail of
    # the synthetic length distribution); the KV cache is a paged pool sized by kv_pool_tokens, so
    # the window costs nothing until a long prompt uses it (prompts were truncated at 2k)
    max_seq: int = 16384
    kv_pool_tokens: int = 0  # 0 = max_batch x 4096 tokens (or max_seq, whichever is larger)
    tokenizer: str = ""
    checkpoint: str = ""
    request_timeout: float = 120.0
    num_retries: int = 3
    # fine-tuning
    model: str = "tiny"  # preset name, or a Hugging Face Llama directory (config.json + safetensors)
    finetune: str = "lora"  # lora | full
    parallel: str = "ddp"  # ddp | zero1 (sharded optimizer) | zero3 (sharded everything)
    sequence_parallel: int = 1  # Ulysses SP degree (ranks per sequence); world = dp x sp
    context_parallel: int = 1  # ring-attention CP degree (zigzag sequence shards); world = dp x cp
    lora_r: int = 16
    lora_alpha: float = 32.0
    lr: float = 1e-4
    weight_decay: float = 0.0
    grad_clip: float = 1.0
    warmup_steps: int = 0
    steps: int = 0  # 0 = run epochs over the dataset
    seq_len: int = 512
    micro_batch: int = 4
    grad_accum: int = 1
    bucket_mb: float = 128.0
    activation_checkpointing: bool = False
    ckpt_layers: int = -1  # with activation_checkpointing: -1 = every layer, N = only the first N (selective)
    ckpt_dir: str = ""
    save_every: int = 0
    save_hf: str = ""  # at the end: write the model as a Hugging Face Llama directory (LoRA merged)
    resume: bool = True
    log_every: int = 10
    metrics_file: str = ""
    gpu_monitor_s: float = 0.0  # AMD SMI sampling period into the metrics file (0 = off)
    check_sync_every: int = 0  # desync check of DDP replicas: 0 = once after init/resume, N = also every N steps, -1 = off
    profile_ranges: bool = True  # roctx ranges around train-step phases (rocprofv3 --marker-trace)
    # inference driver: opt-in gather of every rank's results to rank 0
    gather_results: bool = False
    results_file: str = ""  # rank 0 writes the gathered records as JSONL
    # fault injection (tests / drills)
    fault_rank: int = -1
    fault_step: int = -1
    fault_kind: str = ""  # exit | hang | nan | raise


def _coerce(f, v):
    t = f.type if not isinstance(f.type, str) else {"int": int, "float": float, "bool": bool, "str": str}.get(f.type, str)
    if t is bool:
        if isinstance(v, bool):
            return v
        return str(v).lower() in ("1", "true", "yes", "on")
    return t(v)


def load_config(config_dict: dict | None = None, argv: list[str] | None = None, use_env: bool = True) -> RunConfig:
    cfg = RunConfig()
    flds = {f.name: f for f in fields(RunConfig)}
    if config_dict:
        for k, v in config_dict.items():
            name = k.lower()
            if name in flds and v is not None:
                setattr(cfg, name, _coerce(flds[name], v))
    if use_env:
        for name, f in flds.items():
            ev = os.environ.get("MXLLM_" + name.upper())
            if ev is not None:
                setattr(cfg, name, _coerce(f, ev))
    if argv is not None:
        ap = argparse.ArgumentParser(allow_abbrev=False)
        for name, f in flds.items():
            ap.add_argument("--" + name.replace("_", "-"), dest=name, default=None)
        ns, _ = ap.parse_known_args(argv)
        for name, f in flds.items():
            v = getattr(ns, name)
            if v is not None:
                setattr(cfg, name, _coerce(f, v))
    return cfg


def as_dict(cfg: RunConfig) -> dict:
    return dataclasses.asdict(cfg)
