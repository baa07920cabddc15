"""Structured metrics: JSONL step records + rank-aware logging."""
from __future__ import annotations

import json
import logging
import os
import time


def setup_rank_logging(rank: int, level_main=logging.INFO, level_other=logging.WARNING):
    fmt = f"%(asctime)s - [rank {rank}] %(levelname)s - %(message)s"
    logging.basicConfig(level=level_main if rank == 0 else level_other, format=fmt, datefmt="%Y-%m-%d %H:%M:%S")


class MetricsWriter:
    """Append-only JSONL; only rank 0 writes unless ``all_ranks``."""

    def __init__(self, path: str | None, rank: int = 0, all_ranks: bool = False):
        self.path = path if path and (rank == 0 or all_ranks) else None
        self.rank = rank
        if self.path:
            os.makedirs(os.path.dirname(os.path.abspath(self.path)), exist_ok=True)

    def write(self, **rec):
        if not self.path:
            return
        rec.setdefault("ts", time.time())
        rec.setdefault("rank", self.rank)
        with open(self.path, "a") as f:
            f.write(json.dumps(rec) + "\n")
