"""Rank-tagged logging and JSONL metrics.

The reference's only observability is one "Hello world, rank r out of P" printf per rank
(/root/reference/namegensf.cu:365-366) plus CUDA_CALL's stderr line.  Here: a rank-prefixed
logger (rank 0 by default), a JSONL metrics sink, and a wall-clock step timer.
"""
from __future__ import annotations

import json
import os
import sys
import time
from typing import Any, Dict, Optional


def _rank() -> int:
    return int(os.environ.get("RANK", "0"))


def log(msg: str, all_ranks: bool = False, file=None) -> None:
    r = _rank()
    if all_ranks or r == 0:
        print(f"[rank {r}] {msg}", file=file or sys.stderr, flush=True)


class MetricsWriter:
    """Appends one JSON object per record; only rank 0 writes unless all_ranks."""

    def __init__(self, path: Optional[str], all_ranks: bool = False):
        self.path = path
        self.enabled = path is not None and (all_ranks or _rank() == 0)
        if self.enabled:
            os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        self._f = open(path, "a") if self.enabled else None

    def write(self, **rec: Any) -> None:
        if not self._f:
            return
        rec.setdefault("ts", time.time())
        rec.setdefault("rank", _rank())
        self._f.write(json.dumps(rec) + "\n")
        self._f.flush()

    def close(self) -> None:
        if self._f:
            self._f.close()
            self._f = None


class StepTimer:
    """Wall-clock throughput over a window of steps (device-synchronised by the caller)."""

    def __init__(self):
        self.t0 = time.perf_counter()
        self.n = 0

    def tick(self, k: int = 1) -> None:
        self.n += k

    def rate(self) -> Dict[str, float]:
        dt = time.perf_counter() - self.t0
        out = {"seconds": dt, "steps": self.n, "steps_per_s": self.n / dt if dt > 0 else 0.0}
        self.t0, self.n = time.perf_counter(), 0
        return out
