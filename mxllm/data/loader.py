"""Fine-tuning data path: tokenise -> pack -> native threaded loader -> device.

``TokenLoader`` wraps the C++ ``torch.classes.mxllm.TokenLoader``
(csrc/runtime/dataloader.cpp): distributed per-epoch shuffling, background
batch assembly into pinned host memory, exact resume.  ``next_device()``
issues the H2D copy non_blocking on the current stream.
"""
from __future__ import annotations

import torch

from ..ops import _ext


def pack_texts(texts, tokenizer, eos_id: int) -> torch.Tensor:
    docs = [torch.tensor(tokenizer.encode(t), dtype=torch.int32) for t in texts]
    if _ext.available():
        return torch.ops.mxllm.pack_documents(docs, eos_id)
    out = []
    for d in docs:
        out.append(d)
        out.append(torch.tensor([eos_id], dtype=torch.int32))
    return torch.cat(out)


class TokenLoader:
    def __init__(self, tokens: torch.Tensor, seq_len: int, batch: int, rank: int = 0, world: int = 1, seed: int = 0,
                 device=None, depth: int = 4):
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        pin = self.device.type == "cuda"
        if not _ext.available():
            raise RuntimeError("native TokenLoader requires mxllm/_C.so (python -m mxllm._build)")
        need = seq_len + 1
        if tokens.numel() < need * world * batch:  # tiny corpora: repeat the stream
            reps = (need * world * batch + tokens.numel() - 1) // tokens.numel()
            tokens = tokens.repeat(reps)
        self._l = torch.classes.mxllm.TokenLoader(tokens.to(torch.int32).contiguous(), seq_len, batch, rank, world,
                                                  seed, pin, depth)
        self.batches_per_epoch = self._l.batches_per_epoch()

    def next(self):
        ids, lab, epoch, idx = self._l.next()
        return ids, lab, epoch, idx

    def next_device(self):
        ids, lab, epoch, idx = self._l.next()
        nb = self.device.type == "cuda"
        return ids.to(self.device, non_blocking=nb), lab.to(self.device, non_blocking=nb), epoch, idx

    def state(self) -> dict:
        e, c = self._l.state()
        return {"epoch": int(e), "cursor": int(c)}

    def restore(self, st: dict):
        self._l.restore(int(st["epoch"]), int(st["cursor"]))

    def close(self):
        self._l.shutdown()
