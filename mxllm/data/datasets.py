"""Datasets: the reference's ``CustomDataset``, an offline IMDB-like text set,
and synthetic token batches for fine-tuning benchmarks.

Reference: ``CustomDataset`` (src/distributed_inference.py:23-32), data load
``load_dataset("imdb", split="train[:1%]")`` (:56).  The GPU box and this
container have no network, so ``imdb_like`` produces a
deterministic synthetic stand-in with the same schema ({"text", "label"}),
the same row count (250 = 1% of IMDB train) and a review-like length
distribution; ``load_text_dataset`` tries a local HF ``datasets`` cache first.
"""
from __future__ import annotations

import logging
import random

import torch
from torch.utils.data import Dataset

log = logging.getLogger("mxllm.data")


class CustomDataset(Dataset):
    """Map-style dataset over parallel lists -> {"text": str, "label": int}."""

    def __init__(self, texts, labels):
        self.texts = texts
        self.labels = labels

    def __len__(self):
        return len(self.texts)

    def __getitem__(self, idx):
        return {"text": self.texts[idx], "label": self.labels[idx]}


_POS = ["wonderful", "moving", "brilliant", "superb", "charming", "gripping", "heartfelt", "delightful",
        "masterful", "funny", "beautiful", "memorable"]
_NEG = ["dull", "tedious", "awful", "clumsy", "lifeless", "predictable", "boring", "forgettable",
        "painful", "messy", "flat", "disappointing"]
_NOUN = ["film", "movie", "story", "cast", "script", "director", "plot", "soundtrack", "ending", "performance",
         "cinematography", "dialogue", "pacing", "screenplay", "character"]
_FILL = ["the", "a", "this", "that", "and", "but", "with", "was", "is", "really", "quite", "very", "of", "in",
         "I", "it", "so", "just", "an", "at", "on", "for", "me", "my", "we", "they"]


def imdb_like(n_rows: int = 250, seed: int = 0) -> tuple[list[str], list[int]]:
    """Deterministic synthetic movie reviews with binary sentiment labels.
    Lengths are log-normal (median ~ 900 chars, long tail to ~ 8k chars)."""
    rng = random.Random(seed)
    texts, labels = [], []
    for _ in range(n_rows):
        label = rng.randint(0, 1)
        adj = _POS if label else _NEG
        target = int(min(8000, max(60, rng.lognormvariate(6.8, 0.6))))
        words = []
        size = 0
        while size < target:
            r = rng.random()
            w = rng.choice(adj) if r < 0.12 else rng.choice(_NOUN) if r < 0.3 else rng.choice(_FILL)
            words.append(w)
            size += len(w) + 1
            if rng.random() < 0.07:
                words[-1] += "."
        text = " ".join(words)
        texts.append(text[0].upper() + text[1:])
        labels.append(label)
    return texts, labels


def load_text_dataset(name: str = "imdb", split: str = "train[:1%]", n_rows: int = 250, seed: int = 0):
    """(texts, labels): HF ``datasets`` from the local cache if present, else synthetic."""
    if name != "synthetic":
        try:
            import datasets  # noqa: F401
            from datasets import load_dataset

            ds = load_dataset(name, split=split)
            return list(ds["text"]), list(ds["label"])
        except Exception as e:  # noqa: BLE001 — offline / not cached
            log.info("dataset %s unavailable (%s); using synthetic imdb-like data", name, type(e).__name__)
    return imdb_like(n_rows, seed)


class SyntheticTokens:
    """Random-token LM batches of a fixed shape, generated on the device.

    Each row is drawn as seq_len + 1 tokens: ids are the first seq_len, labels
    the next-token targets (the same stream shifted by one), so every position,
    the last included, has a real target (no -100).  Seeded per rank so DDP
    ranks see different data, reproducible across restarts via ``state``.
    """

    def __init__(self, vocab: int, batch: int, seq_len: int, device, seed: int = 0, rank: int = 0):
        self.vocab, self.batch, self.seq_len = vocab, batch, seq_len
        self.device = torch.device(device)
        self.gen = torch.Generator(device=self.device)
        self.seed = seed * 1000003 + rank
        self.gen.manual_seed(self.seed)
        self.step = 0

    def next(self) -> tuple[torch.Tensor, torch.Tensor]:
        stream = torch.randint(0, self.vocab, (self.batch, self.seq_len + 1), generator=self.gen,
                               device=self.device)
        self.step += 1
        ids = stream[:, :-1].contiguous()
        labels = stream[:, 1:].contiguous()
        return ids, labels

    def state(self) -> dict:
        return {"seed": self.seed, "step": self.step}

    def restore(self, st: dict):
        self.gen.manual_seed(st["seed"])
        self.step = 0
        for _ in range(st["step"]):
            self.next()
