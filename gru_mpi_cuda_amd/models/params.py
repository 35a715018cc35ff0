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


# ------------------------------------------------------------------ padding to the MFMA tile grid
# The HIP engine tiles V, E and H by 64.  Other sizes run on a zero-padded model, which is exact:
# padded hidden units have zero weights and biases, so from h0 = 0 they stay 0 (r = z = 1/2,
# n = tanh 0 = 0), contribute nothing to real units, and receive zero gradient (their dy and
# dh are zero); padded embedding columns are zero on both sides of W_ih0; padded vocabulary rows
# get a logit bias of MASKED_LOGIT, i.e. softmax probability exactly 0 and zero gradient, so Adam
# never moves any padded entry.
MASKED_LOGIT = -30000.0
PAD_MULT = 64


def _round_up(n: int, m: int) -> int:
    return (n + m - 1) // m * m


def pad_config(cfg: GRUConfig, mult: int = PAD_MULT) -> GRUConfig:
    return cfg.replace(vocab=_round_up(cfg.vocab, mult), embed=_round_up(cfg.embed, mult),
                       hidden=_round_up(cfg.hidden, mult))


def pad_params(params: Dict[str, torch.Tensor], cfg: GRUConfig, pcfg: GRUConfig,
               masked_bias: bool = True) -> Dict[str, torch.Tensor]:
    """cfg-shaped tensors -> pcfg-shaped (zero padding per gate block; masked_bias=False pads the
    FC bias with zeros too, for optimiser moments)."""
    H, Hp = cfg.hidden, pcfg.hidden
    out: Dict[str, torch.Tensor] = {}
    for k, v in params.items():
        shp = param_shapes(pcfg)[k]
        if k.startswith(("weight_ih_l", "weight_hh_l")):
            l = int(k.rsplit("l", 1)[1])
            inn = cfg.layer_in(l) if k.startswith("weight_ih") else H
            innp = pcfg.layer_in(l) if k.startswith("weight_ih") else Hp
            p = v.new_zeros(3, Hp, innp)
            p[:, :H, :inn] = v.reshape(3, H, inn)
            out[k] = p.reshape(shp)
        elif k.startswith(("bias_ih_l", "bias_hh_l")):
            p = v.new_zeros(3, Hp)
            p[:, :H] = v.reshape(3, H)
            out[k] = p.reshape(shp)
        elif k == "fc.bias":
            p = v.new_full(shp, MASKED_LOGIT if masked_bias else 0.0)
            p[:cfg.vocab] = v
            out[k] = p
        else:   # embedding [V][E], fc.weight [V][H]
            p = v.new_zeros(shp)
            p[:v.shape[0], :v.shape[1]] = v
            out[k] = p
    return out


def unpad_params(params: Dict[str, torch.Tensor], cfg: GRUConfig, pcfg: GRUConfig) -> Dict[str, torch.Tensor]:
    """pcfg-shaped tensors -> cfg-shaped (the real entries)."""
    H, Hp = cfg.hidden, pcfg.hidden
    out: Dict[str, torch.Tensor] = {}
    for k, v in params.items():
        if k.startswith(("weight_ih_l", "weight_hh_l")):
            l = int(k.rsplit("l", 1)[1])
            inn = cfg.layer_in(l) if k.startswith("weight_ih") else H
            innp = pcfg.layer_in(l) if k.startswith("weight_ih") else Hp
            out[k] = v.reshape(3, Hp, innp)[:, :H, :inn].reshape(3 * H, inn).contiguous()
        elif k.startswith(("bias_ih_l", "bias_hh_l")):
            out[k] = v.reshape(3, Hp)[:, :H].reshape(3 * H).contiguous()
        elif k == "fc.bias":
            out[k] = v[:cfg.vocab].contiguous()
        else:
            out[k] = v[:param_shapes(cfg)[k][0], :param_shapes(cfg)[k][1]].contiguous()
    return out
