"""Synthetic name data (BASELINE.json: "synthetic name sequences / random-init weights").

There is no dataset in the reference (it only *generates*, namegensf.cu:627-890) and
no network here, so training data is a deterministic, seeded syllable generator.
Names are byte strings (char id = byte value, V = 256 as NUM_CHAR, namegensf.cu:862).

Batches are *packed*: ``SOS name EOS SOS name EOS ...`` streams cut into windows of
T+1 ids, so every position of a [B, T] batch is a valid next-char target (no
padding waste in the timed benchmark).  ``make_padded_batch`` gives the
one-name-per-row form (ignore label -1 after EOS) used by tests/CLI.
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import numpy as np

_ONSETS = ["", "b", "br", "c", "ch", "d", "dr", "f", "g", "gr", "h", "j", "k", "kr", "l",
           "m", "n", "p", "r", "s", "sh", "st", "t", "th", "tr", "v", "w", "y", "z"]
_VOWELS = ["a", "e", "i", "o", "u", "ae", "ai", "ia", "io", "ou", "y", "ee"]
_CODAS = ["", "", "", "n", "r", "l", "s", "th", "m", "nd", "x", "k"]


def synthetic_names(n: int, seed: int = 0, max_len: int = 10) -> List[bytes]:
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        syl = int(rng.integers(1, 4))
        s = "".join(_ONSETS[rng.integers(len(_ONSETS))] + _VOWELS[rng.integers(len(_VOWELS))]
                    + _CODAS[rng.integers(len(_CODAS))] for _ in range(syl))
        s = s[: max(1, max_len - 1)].capitalize()
        out.append(s.encode())
    return out


class NameStream:
    """Endless packed stream of synthetic names -> [B, T] (inputs, labels) int32 arrays."""

    def __init__(self, batch: int, seq: int, sos: int = 0, eos: int = 0, seed: int = 0,
                 max_len: int = 10):
        self.B, self.T, self.sos, self.eos, self.max_len = batch, seq, sos, eos, max_len
        self._seed = seed
        self._k = 0
        self._buf = np.zeros(0, dtype=np.int32)

    def _refill(self, need: int) -> None:
        chunks = [self._buf]
        have = self._buf.size
        while have < need:
            names = synthetic_names(4096, seed=self._seed * 1_000_003 + self._k, max_len=self.max_len)
            self._k += 1
            ids = []
            for nm in names:
                ids.append(self.sos)
                ids.extend(nm)
                ids.append(self.eos)
            a = np.asarray(ids, dtype=np.int32)
            chunks.append(a)
            have += a.size
        self._buf = np.concatenate(chunks)

    def next(self) -> Tuple[np.ndarray, np.ndarray]:
        B, T = self.B, self.T
        need = B * (T + 1)
        if self._buf.size < need:
            self._refill(need)
        win = self._buf[:need].reshape(B, T + 1)
        self._buf = self._buf[need:]
        return np.ascontiguousarray(win[:, :T]), np.ascontiguousarray(win[:, 1:])


class NativeNameStream:
    """``NameStream`` interface over the native loader (csrc/data/name_loader.cpp): a C++ producer
    thread packs names into [B, T] batches ahead of the training loop (the Python generator above
    costs ~20 ms per 256 x 33 batch, 80x one training step).  ``path``: a names file, one name
    per line, reshuffled every epoch; default: the synthetic syllable generator (same tables, its
    own seeded stream)."""

    def __init__(self, batch: int, seq: int, sos: int = 0, eos: int = 0, seed: int = 0,
                 max_len: int = 10, path: Optional[str] = None, prefetch: int = 4):
        from ..ops import load_ext
        self.B, self.T = batch, seq
        self._L = load_ext(build_if_missing=False).NameLoader(dict(B=batch, T=seq, sos=sos, eos=eos, seed=seed, max_len=max_len,
                                             prefetch=prefetch, path=path or ""))

    def next(self) -> Tuple[np.ndarray, np.ndarray]:
        return self._L.next(self.B, self.T)

    @property
    def epoch(self) -> int:
        return self._L.epoch()


def make_stream(batch: int, seq: int, sos: int = 0, eos: int = 0, seed: int = 0, max_len: int = 10,
                path: Optional[str] = None, native: bool = True):
    """The training loop's data source: the native prefetching loader when the extension is
    built, else the Python generator (files need the native loader)."""
    if native:
        from ..ops._ext import StaleExtensionError
        try:
            return NativeNameStream(batch, seq, sos, eos, seed, max_len, path)
        except StaleExtensionError:
            raise   # a stale build must fail loudly here too, not fall back to the Python stream
        except (ImportError, OSError, AttributeError):
            if path:
                raise
    if path:
        raise RuntimeError("a names file needs the native loader (python -m gru_mpi_cuda_amd.build_ext)")
    return NameStream(batch, seq, sos, eos, seed, max_len)


def make_padded_batch(names: List[bytes], seq: int, sos: int = 0, eos: int = 0
                      ) -> Tuple[np.ndarray, np.ndarray]:
    """One name per row: x = [SOS, c1..], y = [c1.., EOS, -1...] (label -1 = ignore)."""
    B = len(names)
    x = np.zeros((B, seq), dtype=np.int32)
    y = np.full((B, seq), -1, dtype=np.int32)
    for i, nm in enumerate(names):
        ids = [sos] + list(nm[: seq - 1]) + [eos]
        n = min(len(ids) - 1, seq)
        x[i, :n] = ids[:n]
        x[i, n:] = eos
        y[i, :n] = ids[1:n + 1]
    return x, y


def random_floats(n: int, max_len: int, seed: int = 0) -> np.ndarray:
    """The reference's external uniform randoms, N*MAX_LEN floats in [0,1) (namegensf.cu:315-321)."""
    return np.random.default_rng(seed).random(n * max_len, dtype=np.float32)
