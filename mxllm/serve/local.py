"""Build and register the in-process engine that answers ``completion()`` calls
when ``API_BASE`` is "local" (the default) — the model is served from this
rank's own GPU instead of the reference's remote API."""
from __future__ import annotations

import logging

import torch

from . import client
from .engine import Engine

log = logging.getLogger("mxllm.local")


def preset_for(model_name: str, device: torch.device) -> str:
    n = (model_name or "").lower()
    if "tiny" in n:
        return "tiny"
    if device.type != "cuda":
        return "tiny"  # CPU plumbing runs: tiny random-init stub (BASELINE config 1)
    for key, preset in (("70b", "llama3.1-70b"), ("8b", "llama3.1-8b"), ("1b", "llama3.2-1b")):
        if key in n:
            return preset
    return "tiny"


def ensure_local_engine(model_name: str, device, engine_model: str = "", max_batch: int = 8, max_seq: int = 16384,
                        tokenizer_path: str = "", checkpoint: str = "", seed: int = 0, weights: str = "bf16",
                        kv_pool_tokens: int = 0):
    """Build (once per model name) and register the local engine.  The KV cache is a paged
    pool of ``kv_pool_tokens`` (0: max(max_batch x 4096, max_seq)) shared by every slot, so a
    long context window costs HBM only when a long prompt is admitted; prompts are cut to
    ``max_seq - 64`` tokens (left-truncation) only beyond the window."""
    from ..data.tokenizer import get_tokenizer
    from ..models import build_model, tokenizer_path_for

    if model_name in client._LOCAL:
        return client._LOCAL[model_name]
    device = torch.device(device)
    # a preset name, or a Hugging Face Llama directory (real weights + its tokenizer.json)
    preset = engine_model or preset_for(model_name, device)
    log.info("local engine: %s (%s) on %s", model_name, preset, device)
    model = build_model(preset, device=device, seed=seed)
    cfg = model.cfg
    tokenizer_path = tokenizer_path_for(preset, tokenizer_path)
    if checkpoint:
        from ..train.checkpoint import load_model_weights

        load_model_weights(model, checkpoint)
    model.eval()
    if weights == "fp8":
        from .quant import quantize_model_fp8_

        quantize_model_fp8_(model)
    tok = get_tokenizer(cfg.vocab_size, tokenizer_path or None, cfg.bos_id, cfg.eos_id)
    max_seq = min(max_seq, cfg.max_seq_len)
    pool = kv_pool_tokens or max(max_batch * 4096, max_seq)
    eng = Engine(model, max_batch=max_batch, max_seq=max_seq, eos_ids=(cfg.eos_id,), kv_pool_tokens=pool)
    client.register_local(model_name, eng, _Truncating(tok, max_seq - 64))
    return client._LOCAL[model_name]


class _Truncating:
    """Keeps prompts inside the engine's context window (left-truncation)."""

    def __init__(self, tok, max_prompt: int):
        self.tok, self.max_prompt = tok, max(16, max_prompt)
        self.eos_id = getattr(tok, "eos_id", None)

    def apply_chat_template(self, messages):
        ids = self.tok.apply_chat_template(messages)
        return ids[-self.max_prompt:]

    def encode(self, text, bos=True):
        return self.tok.encode(text, bos)[-self.max_prompt:]

    def decode(self, ids):
        return self.tok.decode(ids)
