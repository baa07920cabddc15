"""Tokenizers.

* ``ByteTokenizer`` — offline, dependency-free UTF-8 byte-level tokenizer
  (ids 0..255 = bytes, 256 = BOS, 257 = EOS, padded up to the model vocab).
* ``HFTokenizer`` — wraps a local ``tokenizer.json`` (Llama-3 BPE) via the
  ``tokenizers`` package when one is on disk.  No downloads ever.
"""
from __future__ import annotations

import os


class ByteTokenizer:
    def __init__(self, vocab_size: int = 512, bos_id: int = 256, eos_id: int = 257):
        self.vocab_size = vocab_size
        self.bos_id = bos_id if bos_id < vocab_size else 256
        self.eos_id = eos_id if eos_id < vocab_size else 257

    def encode(self, text: str, bos: bool = True) -> list[int]:
        ids = list(text.encode("utf-8", errors="replace"))
        return ([self.bos_id] if bos else []) + ids

    def decode(self, ids) -> str:
        return bytes([i for i in ids if 0 <= i < 256]).decode("utf-8", errors="replace")

    def apply_chat_template(self, messages: list[dict]) -> list[int]:
        parts = []
        for m in messages:
            parts.append(f"<|{m.get('role', 'user')}|>\n{m.get('content', '')}\n")
        parts.append("<|assistant|>\n")
        return self.encode("".join(parts))


class HFTokenizer:
    def __init__(self, path: str):
        from tokenizers import Tokenizer

        self.tok = Tokenizer.from_file(path)
        self.vocab_size = self.tok.get_vocab_size()
        self.bos_id = self.tok.token_to_id("<|begin_of_text|>") or 128000
        self.eos_id = self.tok.token_to_id("<|eot_id|>") or 128009

    def encode(self, text: str, bos: bool = True) -> list[int]:
        ids = self.tok.encode(text, add_special_tokens=False).ids
        return ([self.bos_id] if bos else []) + ids

    def decode(self, ids) -> str:
        return self.tok.decode(list(ids))

    def apply_chat_template(self, messages: list[dict]) -> list[int]:
        s = "<|begin_of_text|>"
        for m in messages:
            s += f"<|start_header_id|>{m.get('role', 'user')}<|end_header_id|>\n\n{m.get('content', '')}<|eot_id|>"
        s += "<|start_header_id|>assistant<|end_header_id|>\n\n"
        return self.tok.encode(s, add_special_tokens=False).ids


def get_tokenizer(vocab_size: int, path: str | None = None, bos_id: int = 256, eos_id: int = 257):
    path = path or os.environ.get("MXLLM_TOKENIZER")
    if path and os.path.exists(path):
        return HFTokenizer(path)
    return ByteTokenizer(vocab_size, bos_id if bos_id < 258 else 256, eos_id if eos_id < 258 else 257)
