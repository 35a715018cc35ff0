"""Generation engines + the reference's 3-call API.

``HipGenerator`` drives the native device-resident generator (csrc/engine/generator.cpp).
``namegen_initialize / namegen / namegen_finalize`` keep the reference's signatures and
semantics (/root/reference/namegensf.cu:359, 627, 897):

* every rank generates a contiguous slice of the N names (remainder spread over the first
  ranks instead of dropped), each name n consuming the *global*
  ``random_floats[n*MAX_LEN + l]`` at step l, so the output is independent of world size
  (the §3.2 invariant);
* rank 0 ends with ``output[N*(MAX_LEN+1)]``: each name's chars, the EOS char written before
  stopping, NUL padding;
* only rank 0 reads the parameter file; weights are broadcast.

Collectives: RCCL all-gather of the fixed-size per-rank output slabs on device (replaces
MPI_Scatter of the randoms + MPI_Gather of the names, namegensf.cu:636,889); the randoms
are not scattered at all -- every rank reads only its own slice of the caller's array.
"""
from __future__ import annotations

from typing import Dict, Optional

import numpy as np
import torch

from ..config import GRUConfig
from ..models import cpu_ref
from ..models.params import flat_layout, pad_config, pad_params, to_flat
from ..parallel.dist import DistCtx, shard


PRECISIONS = ("fp32", "bf16", "bf16x3")
_MODE = {"bf16": 0, "fp32": 1, "bf16x3": 2}   # GenDims::fp32


class HipGenerator:
    """precision "fp32" (default): the reference's arithmetic (namegensf.cu:233-242, 294-333) --
    fp32 MFMA GEMMs on the fp32 master weights, IEEE gates and softmax;
    "bf16x3": the same with its products as bf16 MFMA GEMMs over split operands (x = hi + lo,
    hi*hi + hi*lo + lo*hi in fp32: ~2^-16 relative error per product, 1.9x the fp32 speed at 4096
    names).  Opt-in: 2400 names (profiles/r3_gen_default_decision.jsonl) matched the fp64 oracle
    as often as fp32, but that sample cannot separate a 2^-16 product error from fp32 on near-tie
    samples (parity unpinned);
    "bf16": bf16 MFMA fast mode (fused step kernels, bf16 weight copies).
    Small batches run the exact fp32 persistent kernel in both fp32 modes."""

    def __init__(self, cfg: GRUConfig, params: Dict[str, torch.Tensor], max_batch: int = 4096,
                 device: Optional[torch.device] = None, flat: Optional[torch.Tensor] = None,
                 precision: str = "fp32"):
        if precision not in PRECISIONS:
            raise ValueError(f"precision must be one of {PRECISIONS}")
        self.precision = precision
        from ..ops import load_ext
        self.C = load_ext()
        self.cfg = cfg
        self.dev = device or torch.device("cuda", torch.cuda.current_device())
        # E, H off the 64-grid: the exactly equivalent zero-padded model (models/params.py).  The
        # vocabulary is not padded: the sampler's fallback index is V - 1 (namegensf.cu:333)
        if cfg.vocab % 64:
            raise ValueError(f"HIP generator needs vocab % 64 == 0 (got {cfg.vocab})")
        icfg = pad_config(cfg).replace(vocab=cfg.vocab)
        if icfg != cfg:
            if flat is not None:
                raise ValueError("a shared flat buffer needs embed and hidden to be multiples of 64")
            params = pad_params(params, cfg, icfg)
        self.layout = flat_layout(icfg)
        self.flat = flat if flat is not None else to_flat(icfg, params).to(self.dev)
        offsets = {s.name: s.offset for s in self.layout.segments}
        dims = dict(V=cfg.vocab, E=icfg.embed, H=icfg.hidden, L=cfg.layers, max_len=cfg.max_len,
                    sos=cfg.sos, eos=cfg.eos, max_batch=max_batch, fp32=_MODE[precision])
        self.g = self.C.Generator(dims, self.flat.data_ptr(), offsets)
        self.g.refresh_weights(self._s())

    def _s(self) -> int:
        return torch.cuda.current_stream(self.dev).cuda_stream

    def generate_device(self, rf_dev: torch.Tensor, n: int) -> torch.Tensor:
        ML = self.cfg.max_len
        out = torch.empty(max(n, 1), ML + 1, dtype=torch.uint8, device=self.dev)   # every row written
        if n > 0:
            self.g.generate(rf_dev.data_ptr(), n, out.data_ptr(), self._s())
        return out[:n]

    def generate(self, rfloats: np.ndarray, start: int = 0, count: Optional[int] = None) -> np.ndarray:
        ML = self.cfg.max_len
        N = (rfloats.size // ML - start) if count is None else count
        rf = torch.from_numpy(np.ascontiguousarray(rfloats[start * ML:(start + N) * ML], dtype=np.float32))
        rf = rf.to(self.dev)
        return self.generate_device(rf, N).cpu().numpy()


# --------------------------------------------------------------------------- 3-call API
class _State:
    cfg: GRUConfig
    ctx: DistCtx
    gen = None            # HipGenerator or None (CPU path)
    params = None
    comm = None


_S: Optional[_State] = None


def namegen_initialize(N: int, rng_seed: int, parameter_fname: str, cfg: Optional[GRUConfig] = None,
                       fmt: str = "auto", ctx: Optional[DistCtx] = None, precision: str = "fp32") -> None:
    """namegensf.cu:359-618.  ``rng_seed`` is accepted and unused, as in the reference.
    ``precision``: "fp32" (default), "bf16x3" (split-bf16 products) or "bf16" (fast mode) on the GPU
    path (see HipGenerator); the CPU path is the fp32 oracle."""
    global _S
    from ..parallel import dist as gdist
    from ..utils import ckpt
    s = _State()
    s.ctx = ctx or gdist.init(verbose=True)
    if s.ctx.is_main:
        s.cfg, params = ckpt.load(parameter_fname, cfg, fmt)
    else:
        s.cfg, params = (cfg or GRUConfig()), None
    if s.ctx.world > 1:   # dims + weights from rank 0
        import torch.distributed as dist
        box = [s.cfg]
        dist.broadcast_object_list(box, 0)
        s.cfg = box[0]
    if s.ctx.device.type == "cuda":
        from ..parallel.rccl import make_comm
        s.comm = make_comm(s.ctx)
        lay = flat_layout(s.cfg)
        flat = (to_flat(s.cfg, params) if params is not None
                else torch.zeros(lay.total)).to(s.ctx.device)
        if s.comm is not None:
            s.comm.broadcast_f32(flat.data_ptr(), lay.total, 0, torch.cuda.current_stream().cuda_stream)
        s.gen = HipGenerator(s.cfg, {}, device=s.ctx.device, flat=flat,
                             max_batch=max(64, min(8192, N // max(1, s.ctx.world) + 1)), precision=precision)
    else:
        lay = flat_layout(s.cfg)
        flat = to_flat(s.cfg, params) if params is not None else torch.zeros(lay.total)
        if s.ctx.world > 1:
            import torch.distributed as dist
            dist.broadcast(flat, 0)
        s.params = {k: v.clone() for k, v in lay.views(flat).items()}
    gdist.barrier()
    _S = s


def namegen(N: int, random_floats: np.ndarray, output: np.ndarray) -> None:
    """namegensf.cu:627-890.  ``output`` (rank 0): uint8 [N*(MAX_LEN+1)] filled in place."""
    assert _S is not None, "call namegen_initialize first"
    cfg, ctx = _S.cfg, _S.ctx
    ML = cfg.max_len
    start, count = shard(N, ctx.rank, ctx.world)
    per = -(-N // ctx.world)          # ceil: fixed slab size for the all-gather
    if _S.gen is not None:
        _S.gen.g.set_global_names(N)   # bf16 mode: the same arithmetic path at every world size
        mine = _S.gen.generate(random_floats, start, count)
        if ctx.world > 1:
            dev = ctx.device
            slab = torch.zeros(per, ML + 1, dtype=torch.uint8, device=dev)
            slab[:count] = torch.from_numpy(mine).to(dev)
            allv = torch.empty(ctx.world, per, ML + 1, dtype=torch.uint8, device=dev)
            _S.comm.allgather_u8(slab.data_ptr(), allv.data_ptr(), slab.numel(),
                                 torch.cuda.current_stream().cuda_stream)
            allv = allv.cpu().numpy()
        else:
            allv = mine[None]
    else:
        mine = cpu_ref.generate(_S.params, cfg, random_floats, start, count)
        if ctx.world > 1:
            import torch.distributed as dist
            slab = torch.zeros(per, ML + 1, dtype=torch.uint8)
            slab[:count] = torch.from_numpy(mine)
            bufs = [torch.empty_like(slab) for _ in range(ctx.world)]
            dist.all_gather(bufs, slab)
            allv = torch.stack(bufs).numpy()
        else:
            allv = mine[None]
    if ctx.is_main:
        res = np.zeros((N, ML + 1), dtype=np.uint8)
        for r in range(ctx.world):
            s0, c0 = shard(N, r, ctx.world)
            res[s0:s0 + c0] = allv[r][:c0]
        output.reshape(-1)[: N * (ML + 1)] = res.reshape(-1)


def namegen_finalize() -> None:
    """namegensf.cu:897-1033 (frees everything; no MPI_Finalize here either)."""
    global _S
    _S = None
    if torch.cuda.is_available():
        torch.cuda.synchronize()


def decode_names(output: np.ndarray, N: int, max_len: int) -> list:
    rows = np.asarray(output, dtype=np.uint8).reshape(-1)[: N * (max_len + 1)].reshape(N, max_len + 1)
    return [bytes(r).split(b"\0", 1)[0].decode("latin-1") for r in rows]
