"""Parameter naming, shapes, initialisation and the flat buffer layout.

Names follow torch's ``nn.GRU`` / ``nn.Linear`` convention (gate order r, z, n),
which SURVEY §3.3 / Appendix A verified is exactly the reference's math:
``weight_ih_l{l} = cat(W_ir{l}, W_iz{l}, W_in{l})`` (reference tensors built at
/root/reference/namegensf.cu:375-407).

Two orderings exist:

* **checkpoint order** (``ckpt_order``): the reference's blob order generalised to
  any L -- embedding, all W_i, all W_h, all b_i, all b_h, W_fc, b_fc
  (namegensf.cu:375-407).
* **flat order** (``flat_layout``): the engine's single contiguous fp32 buffer,
  ordered by gradient *readiness* during backprop-through-time (FC first, then
  layers top-down as W_hh, b_hh, b_ih, W_ih, embedding last) so that gradient all-reduce buckets are
  contiguous slices that become ready in order.  Each segment starts at a
  multiple of 64 floats (256 B) so kernels can use 16-byte vector accesses.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Dict, List, Tuple

import torch

from ..config import GRUConfig

ALIGN = 64  # floats


def param_shapes(cfg: GRUConfig) -> Dict[str, Tuple[int, ...]]:
    V, E, H, L = cfg.vocab, cfg.embed, cfg.hidden, cfg.layers
    shapes: Dict[str, Tuple[int, ...]] = {"embedding": (V, E)}
    for l in range(L):
        shapes[f"weight_ih_l{l}"] = (3 * H, cfg.layer_in(l))
        shapes[f"weight_hh_l{l}"] = (3 * H, H)
        shapes[f"bias_ih_l{l}"] = (3 * H,)
        shapes[f"bias_hh_l{l}"] = (3 * H,)
    shapes["fc.weight"] = (V, H)
    shapes["fc.bias"] = (V,)
    return shapes


def ckpt_order(cfg: GRUConfig) -> List[str]:
    L = cfg.layers
    return (["embedding"]
            + [f"weight_ih_l{l}" for l in range(L)]
            + [f"weight_hh_l{l}" for l in range(L)]
            + [f"bias_ih_l{l}" for l in range(L)]
            + [f"bias_hh_l{l}" for l in range(L)]
            + ["fc.weight", "fc.bias"])


def flat_order(cfg: GRUConfig) -> List[str]:
    names = ["fc.weight", "fc.bias"]
    for l in reversed(range(cfg.layers)):
        # biases before W_ih: layer 0's data-parallel bucket ends inside the W_ih0 segment (the
        # engine all-reduces the V x 3H table gradient dP there and derives dW_ih0 / dEmb after)
        names += [f"weight_hh_l{l}", f"bias_hh_l{l}", f"bias_ih_l{l}", f"weight_ih_l{l}"]
    names.append("embedding")
    return names


@dataclass(frozen=True)
class Segment:
    name: str
    offset: int          # in floats
    shape: Tuple[int, ...]

    @property
    def numel(self) -> int:
        return int(math.prod(self.shape))


@dataclass(frozen=True)
class FlatLayout:
    segments: Tuple[Segment, ...]
    total: int           # padded total, in floats

    def __getitem__(self, name: str) -> Segment:
        for s in self.segments:
            if s.name == name:
                return s
        raise KeyError(name)

    def views(self, flat: torch.Tensor) -> Dict[str, torch.Tensor]:
        return {s.name: flat[s.offset:s.offset + s.numel].view(s.shape) for s in self.segments}


def flat_layout(cfg: GRUConfig) -> FlatLayout:
    shapes = param_shapes(cfg)
    segs, off = [], 0
    for name in flat_order(cfg):
        segs.append(Segment(name, off, shapes[name]))
        n = int(math.prod(shapes[name]))
        off += (n + ALIGN - 1) // ALIGN * ALIGN
    return FlatLayout(tuple(segs), off)


def init_params(cfg: GRUConfig, seed: int | None = None) -> Dict[str, torch.Tensor]:
    """Random init with torch's default distributions (fp32, CPU, deterministic)."""
    g = torch.Generator().manual_seed(cfg.seed if seed is None else seed)
    k = 1.0 / math.sqrt(cfg.hidden)
    out: Dict[str, torch.Tensor] = {}
    for name, shape in param_shapes(cfg).items():
        if name == "embedding":
            out[name] = torch.randn(shape, generator=g) * 0.5
        else:
            out[name] = (torch.rand(shape, generator=g) * 2 - 1) * k
    return out


def to_flat(cfg: GRUConfig, params: Dict[str, torch.Tensor], device="cpu") -> torch.Tensor:
    lay = flat_layout(cfg)
    flat = torch.zeros(lay.total, dtype=torch.float32, device=device)
    views = lay.views(flat)
    for name, v in views.items():
        v.copy_(params[name].to(torch.float32))
    return flat


def from_flat(cfg: GRUConfig, flat: torch.Tensor) -> Dict[str, torch.Tensor]:
    return {k: v.detach().clone() for k, v in flat_layout(cfg).views(flat).items()}
