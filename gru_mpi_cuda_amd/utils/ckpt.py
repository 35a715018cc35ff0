"""Checkpoint I/O.

Reference format (``fmt="ref"``): a headerless little-endian fp32 blob, read by the
reference's ``read_binary`` and sliced into 27 tensors at fixed ``OFFSET0..26``
(/root/reference/namegensf.cu:370-407; layout in SURVEY.md Appendix A).  The
reference only *reads*; here both directions exist, for any L (``ckpt_order``
generalises the group ordering: emb, all W_i, all W_h, all b_i, all b_h, W_fc, b_fc).

Generalised format (``fmt="gen"``): the same blob plus a ``<path>.json`` sidecar
holding the dims, so a file is self-describing.  Training resume state (Adam
moments + step) goes to ``<path>.opt.safetensors`` -- nothing here unpickles.

Only rank 0 reads in the distributed engine; the weights are then broadcast
(fixes the reference's every-rank read, namegensf.cu:368-372 / SURVEY §2.7 item 4).
"""
from __future__ import annotations

import json
import os
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch

from ..config import GRUConfig
from ..models.params import ckpt_order, param_shapes

FORMAT_VERSION = 1


def ref_offsets(cfg: GRUConfig) -> List[Tuple[str, int, Tuple[int, ...]]]:
    """(name, float offset, shape) for every tensor, in blob order (= OFFSETk)."""
    shapes = param_shapes(cfg)
    out, off = [], 0
    for name in ckpt_order(cfg):
        out.append((name, off, shapes[name]))
        off += int(np.prod(shapes[name]))
    return out


def blob_floats(cfg: GRUConfig) -> int:
    """V*E + sum_l 3H*in_l + L*3H^2 + 12H (L=2) + V*H + V  (SURVEY Appendix A formula)."""
    name, off, shape = ref_offsets(cfg)[-1]
    return off + int(np.prod(shape))


def reference_split(cfg: GRUConfig, params: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
    """Split torch-named params into the reference's 27 per-gate tensors (L=2 naming)."""
    H = cfg.hidden
    out = {"character_embedding": params["embedding"]}
    for kind, wname, bname in (("i", "weight_ih", "bias_ih"), ("h", "weight_hh", "bias_hh")):
        for l in range(cfg.layers):
            for gi, g in enumerate("rzn"):
                out[f"W_{kind}{g}{l}"] = params[f"{wname}_l{l}"][gi * H:(gi + 1) * H]
                out[f"b_{kind}{g}{l}"] = params[f"{bname}_l{l}"][gi * H:(gi + 1) * H]
    out["W_fc"] = params["fc.weight"]
    out["b_fc"] = params["fc.bias"]
    return out


def save(path: str, cfg: GRUConfig, params: Dict[str, torch.Tensor], fmt: str = "gen",
         opt_state: Optional[Dict[str, torch.Tensor]] = None) -> None:
    parts = [params[n].detach().to("cpu", torch.float32).contiguous().reshape(-1).numpy()
             for n in ckpt_order(cfg)]
    blob = np.concatenate(parts).astype("<f4", copy=False)
    assert blob.size == blob_floats(cfg)
    tmp = path + ".tmp"
    blob.tofile(tmp)
    os.replace(tmp, path)           # atomic w.r.t. readers
    if fmt == "gen":
        meta = {"format": "gru_mpi_cuda_amd", "version": FORMAT_VERSION,
                "vocab": cfg.vocab, "embed": cfg.embed, "hidden": cfg.hidden,
                "layers": cfg.layers, "max_len": cfg.max_len, "sos": cfg.sos, "eos": cfg.eos,
                "order": ckpt_order(cfg)}
        with open(path + ".json", "w") as f:
            json.dump(meta, f, indent=1)
    elif fmt != "ref":
        raise ValueError(f"unknown checkpoint format {fmt!r}")
    if opt_state is not None:
        from safetensors.torch import save_file
        save_file({k: v.detach().to("cpu").contiguous() for k, v in opt_state.items()},
                  path + ".opt.safetensors")


def load(path: str, cfg: Optional[GRUConfig] = None, fmt: str = "auto"
         ) -> Tuple[GRUConfig, Dict[str, torch.Tensor]]:
    """Returns (config, params).  ``fmt='ref'`` needs ``cfg`` (dims are not in the blob)."""
    side = path + ".json"
    if fmt == "auto":
        fmt = "gen" if os.path.exists(side) else "ref"
    if fmt == "gen":
        with open(side) as f:
            meta = json.load(f)
        base = cfg or GRUConfig()
        cfg = base.replace(**{k: meta[k] for k in ("vocab", "embed", "hidden", "layers",
                                                     "max_len", "sos", "eos")})
    elif cfg is None:
        raise ValueError("reference-format checkpoints are headerless: pass cfg")
    blob = np.fromfile(path, dtype="<f4")
    want = blob_floats(cfg)
    if blob.size != want:
        raise ValueError(f"{path}: {blob.size} floats, config expects {want} "
                         f"(V={cfg.vocab} E={cfg.embed} H={cfg.hidden} L={cfg.layers})")
    params = {}
    for name, off, shape in ref_offsets(cfg):
        n = int(np.prod(shape))
        params[name] = torch.from_numpy(blob[off:off + n].copy()).view(shape)
    return cfg, params


def load_opt_state(path: str) -> Optional[Dict[str, torch.Tensor]]:
    p = path + ".opt.safetensors"
    if not os.path.exists(p):
        return None
    from safetensors.torch import load_file
    return load_file(p)
