"""Training engines.

``HipTrainer``  -- the MI355X path: the native executor (csrc/engine/trainer.cpp) runs the
whole forward + softmax-xent + BPTT + weight-gradient step as one hipGraph over two HIP
streams; gradients are then averaged with bucketed RCCL all-reduce on the device (native
communicator) and a fused Adam + bf16-weight-refresh graph finishes the step.

``CpuTrainer``  -- the CPU reference path (BASELINE config #1): same math in PyTorch
(models/cpu_ref.manual_backward), gloo all-reduce for multi-process tests.

Neither has a reference counterpart: the reference is inference-only.
"""
from __future__ import annotations

import math
from typing import Dict, Optional

import numpy as np
import torch

from ..config import GRUConfig
from ..models import cpu_ref
from ..models.params import flat_layout, from_flat, init_params, pad_config, pad_params, to_flat, unpad_params
from ..parallel.dist import DistCtx, allreduce_mean_buckets, bucket_bounds


def _bucket_list(cfg: GRUConfig, total: int):
    lay = flat_layout(cfg)
    bounds = [s.offset for s in lay.segments]
    return bucket_bounds(total, max(1024, int(cfg.bucket_mb * (1 << 20) / 4)), bounds)


class HipTrainer:
    def __init__(self, cfg: GRUConfig, ctx: Optional[DistCtx] = None,
                 params: Optional[Dict[str, torch.Tensor]] = None, comm=None, use_graph: bool = True):
        from ..ops import load_ext
        self.C = load_ext()
        self.cfg = cfg
        self.ctx = ctx or DistCtx(device=torch.device("cuda", torch.cuda.current_device()))
        self.dev = self.ctx.device
        if cfg.batch % self.ctx.world:
            raise ValueError(f"global batch {cfg.batch} not divisible by world size {self.ctx.world}")
        self.local_batch = cfg.batch // self.ctx.world
        # V, E, H off the 64-grid run on the exactly equivalent zero-padded model (params.py);
        # params / grads / m / v below are in the padded (internal) layout, the accessors
        # (state_dict, grad_dict, load_state, opt_state) speak the user's shapes
        self.icfg = pad_config(cfg)
        self.padded = self.icfg != cfg
        self.layout = flat_layout(self.icfg)
        p0 = params if params is not None else init_params(cfg)
        self.params = to_flat(self.icfg, self._pad(p0)).to(self.dev)
        self.grads = torch.zeros_like(self.params)
        self.m = torch.zeros_like(self.params)
        self.v = torch.zeros_like(self.params)
        self.comm = comm
        self.buckets = _bucket_list(self.icfg, self.layout.total)
        offsets = {s.name: s.offset for s in self.layout.segments}
        ic = self.icfg
        dims = dict(V=ic.vocab, E=ic.embed, H=ic.hidden, L=cfg.layers, B=self.local_batch,
                    T=cfg.seq, chunks=cfg.time_chunks, overlap=int(cfg.overlap))
        from ..models.cpu_ref import LR_SCHEDS
        if cfg.lr_sched not in LR_SCHEDS:
            raise ValueError(f"lr_sched must be one of {LR_SCHEDS}, got {cfg.lr_sched!r}")
        opt = dict(lr=cfg.lr, beta1=cfg.beta1, beta2=cfg.beta2, eps=cfg.eps,
                   weight_decay=cfg.weight_decay, clip_norm=cfg.clip_norm,
                   sgd=int(cfg.optimizer == "sgd"), lr_sched=LR_SCHEDS.index(cfg.lr_sched),
                   warmup_steps=cfg.warmup_steps, total_steps=cfg.total_steps, lr_min=cfg.lr_min,
                   keep_grads=int(cfg.keep_grads))
        self.t = self.C.Trainer(dims, opt, self.params.data_ptr(), self.grads.data_ptr(),
                                self.m.data_ptr(), self.v.data_ptr(), self.layout.total, offsets)
        self.t.set_use_graph(use_graph)
        self.t.set_carry(bool(cfg.carry_hidden))
        if self.comm is not None:     # identical replicas: rank 0's weights everywhere
            self.comm.broadcast_f32(self.params.data_ptr(), self.layout.total, 0, self._stream())
            # all-reduce recorded INTO the step graph: readiness-ordered buckets of at least
            # bucket_mb on a comm stream, overlapped with the rest of the backward
            self.t.set_comm(self.comm, [(a, b - a) for a, b in self.buckets],
                            max(1024, int(cfg.bucket_mb * (1 << 20) / 4)))
            if cfg.shard_optim:
                self.t.set_shard_optim(int(cfg.shard_optim))
            self.t.set_dp_pipeline(int(cfg.dp_pipeline))
        self.t.refresh_weights(self._stream())
        self._one_graph = True
        # does the flat gradient buffer hold the last step's full gradient?  Not after a one-graph
        # step() / steps() without cfg.keep_grads: the fused Adam then sums the split-K / row-block
        # partials in registers and never writes them back (and in data-parallel mode the W_ih0 slot
        # holds the all-reduced dP) -- grad_dict() refuses instead of returning stale values
        self._grads_valid = False
        # host thread watching each launched step, the communicator and the step
        # error word (a persistent kernel's spin limit: that step's update is skipped on device)
        wd = int(cfg.watchdog_ms)
        if wd == -1:
            wd = 120_000 if self.ctx.world > 1 else 0
        if wd >= 0:
            self.t.enable_watchdog(wd)

    def _pad(self, params: Dict[str, torch.Tensor], masked_bias: bool = True) -> Dict[str, torch.Tensor]:
        return pad_params(params, self.cfg, self.icfg, masked_bias) if self.padded else params

    def _unpad(self, params: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
        return unpad_params(params, self.cfg, self.icfg) if self.padded else params

    def check_watchdog(self) -> None:
        """Raise if the watchdog fired (step timeout, RCCL async error or step error word)."""
        if self.t.watchdog_status():
            raise RuntimeError(f"watchdog: {self.t.watchdog_message()}")

    def _stream(self) -> int:
        return torch.cuda.current_stream(self.dev).cuda_stream

    def forward_backward(self, x: np.ndarray, y: np.ndarray) -> None:
        s = self._stream()
        self.t.set_batch(x, y, s)
        self.t.forward_backward(s)
        self._grads_valid = True

    def allreduce_grads(self) -> None:
        if self.comm is None:
            return
        s = self._stream()
        base = self.grads.data_ptr()
        for a, b in self.buckets:
            self.comm.allreduce_avg_f32(base + 4 * a, b - a, s)
        # the step error word, max over ranks: a step that failed anywhere is skipped everywhere
        self.comm.allreduce_max_u32(self.t.buffer("err"), 1, s)

    def optimizer_step(self) -> None:
        self.t.optimizer_step(self._stream())

    def step(self, x: np.ndarray, y: np.ndarray) -> None:
        """Whole step = one hipGraph replay: batch prep, forward, softmax-xent, BPTT, weight
        gradients, bucketed RCCL all-reduce (if data-parallel) and Adam + bf16 weight refresh.
        The flat gradient buffer (grad_dict) holds the step's gradient afterwards only with
        ``cfg.keep_grads``; otherwise grad_dict() raises until the next forward_backward()."""
        s = self._stream()
        self.t.set_batch(x, y, s)
        self.check_watchdog()
        if self._one_graph:
            try:
                self.t.step(s)
                self._grads_valid = bool(self.cfg.keep_grads)
                return
            except RuntimeError as e:   # e.g. RCCL refusing stream capture: fall back, loudly
                if self.comm is None:
                    raise
                import sys
                print(f"[gru_mpi_cuda_amd] in-graph all-reduce unavailable ({e}); "
                      "falling back to per-phase launches", file=sys.stderr)
                self._one_graph = False
                self.t.set_comm(None, [], 1)
        self.t.forward_backward(s)
        self.allreduce_grads()
        self.t.optimizer_step(s)
        self._grads_valid = True

    def steps(self, batches) -> None:
        """len(batches) whole steps as ONE graph launch (Trainer::set_graph_steps): the graph boundary
        (~13 us at the headline) is paid once per group.  Each batch is an (x, y) pair of [B, T]."""
        n = len(batches)
        if n == 1 or not self._one_graph:
            for x, y in batches:
                self.step(x, y)
            return
        if self.t.graph_steps() != n:
            self.t.set_graph_steps(n)
        s = self._stream()
        self.t.set_batches(np.stack([np.asarray(x) for x, _ in batches]), np.stack([np.asarray(y) for _, y in batches]))
        self.check_watchdog()
        try:
            self.t.step_group(s)
            self._grads_valid = bool(self.cfg.keep_grads)
        except RuntimeError as e:   # e.g. a collective refusing capture: one graph per step, loudly
            import sys
            print(f"[gru_mpi_cuda_amd] multi-step graph unavailable ({e}); one graph per step", file=sys.stderr)
            self.t.set_graph_steps(1)
            for x, y in batches:
                self.step(x, y)

    def loss(self) -> float:
        return self.t.read_loss()

    def reset_state(self) -> None:
        """Zero the carried hidden state (truncated BPTT, ``cfg.carry_hidden``)."""
        self.t.reset_hidden(self._stream())

    def comm_stats(self) -> Dict[str, float]:
        """Gradient-collective observability: bytes all-reduced per step inside the
        step graph, and the time of the same collectives run on their own (a probe: it re-reduces
        the gradient buffer after the step, whose Adam update has already consumed it)."""
        if self.comm is None:
            return {}
        log = self.t.allreduce_log() or [(a, b - a) for a, b in self.buckets]
        nbytes = 4 * sum(n for _, n in log)
        s = torch.cuda.current_stream(self.dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        base = self.grads.data_ptr()
        for off, n in log:
            if off >= 0:
                self.comm.allreduce_avg_f32(base + 4 * off, n, s.cuda_stream)
        e1.record(s)
        e1.synchronize()
        return {"allreduce_mb_per_step": nbytes / 2 ** 20, "allreduce_collectives": len(log),
                "allreduce_ms_standalone": e0.elapsed_time(e1)}

    def state_dict(self) -> Dict[str, torch.Tensor]:
        if self.t.shard_mode() == 2:   # other ranks' fp32 master slices are only current after a gather
            self.t.gather_params(self._stream())
        torch.cuda.synchronize(self.dev)
        return self._unpad({k: v.cpu() for k, v in from_flat(self.icfg, self.params).items()})

    def grad_dict(self) -> Dict[str, torch.Tensor]:
        """The last forward_backward()'s gradient (or the last step()'s with ``cfg.keep_grads``)."""
        if not self._grads_valid:
            raise RuntimeError("grad_dict(): the gradient buffer does not hold the last step's gradient "
                               "(one-graph step() without keep_grads: the fused optimiser never writes it "
                               "back); set GRUConfig.keep_grads=True or call forward_backward()")
        torch.cuda.synchronize(self.dev)
        return self._unpad({k: v.cpu() for k, v in from_flat(self.icfg, self.grads).items()})

    def load_state(self, params: Dict[str, torch.Tensor]) -> None:
        self.params.copy_(to_flat(self.icfg, self._pad(params)).to(self.dev))
        self.t.refresh_weights(self._stream())

    def opt_state(self):
        """Adam moments as flat fp32 tensors in the user config's layout (checkpoints).  Sharded
        optimiser: every rank first all-gathers the moment slices the other ranks own."""
        if self.t.shard_optim():
            self.t.gather_opt_state(self._stream())
        torch.cuda.synchronize(self.dev)
        return tuple(to_flat(self.cfg, self._unpad(from_flat(self.icfg, t.cpu()))) for t in (self.m, self.v))

    def load_opt_state(self, m: torch.Tensor, v: torch.Tensor) -> None:
        for dst, src in ((self.m, m), (self.v, v)):
            dst.copy_(to_flat(self.icfg, self._pad(from_flat(self.cfg, src.float()), masked_bias=False)).to(self.dev))


class CpuTrainer:
    def __init__(self, cfg: GRUConfig, ctx: Optional[DistCtx] = None,
                 params: Optional[Dict[str, torch.Tensor]] = None, dtype=torch.float32, bf16_weights: bool = False):
        self.cfg = cfg
        self.ctx = ctx or DistCtx()
        if cfg.batch % self.ctx.world:
            raise ValueError(f"global batch {cfg.batch} not divisible by world size {self.ctx.world}")
        self.local_batch = cfg.batch // self.ctx.world
        p = params if params is not None else init_params(cfg)
        self.layout = flat_layout(cfg)
        self.flat_p = to_flat(cfg, p).to(dtype)
        self.flat_g = torch.zeros_like(self.flat_p)
        self.params = self.layout.views(self.flat_p)
        self.gviews = self.layout.views(self.flat_g)
        if self.ctx.world > 1:          # identical replicas
            import torch.distributed as dist
            dist.broadcast(self.flat_p, 0)
        self.shard = None
        # bf16 working copies (cfg.shard_optim == 2, or bf16_weights=True for its replicated reference):
        # the forward / backward use bf16-rounded weight matrices and fp32 biases, as the device step does
        self.bf16 = bool(bf16_weights) or int(cfg.shard_optim) == 2
        self.flat_bf = None
        if cfg.shard_optim and self.ctx.world > 1:
            # ZeRO-1 twin of Trainer::set_shard_optim: rank r owns flat floats [r*c, (r+1)*c) with c a
            # multiple of 4; the tail past world*c is updated by every rank
            if cfg.clip_norm > 0:
                raise ValueError("shard_optim: gradient clipping is not supported with a sharded optimiser")
            W, r, n = self.ctx.world, self.ctx.rank, self.layout.total
            c = n // (4 * W) * 4
            self.shard = (c, {"own": slice(r * c, (r + 1) * c), "tail": slice(W * c, n)})
            self.opt = cpu_ref.Adam(cfg, {k: self.flat_p[sl] for k, sl in self.shard[1].items()})
            if int(cfg.shard_optim) == 2:   # the gathered flat bf16 working copy (Trainer::pbf_)
                self.flat_bf = self.flat_p.to(torch.bfloat16)
                self._bias_ranges = [(s.offset, s.offset + int(np.prod(s.shape))) for s in self.layout.segments
                                     if "bias" in s.name]
        else:
            self.opt = cpu_ref.Adam(cfg, self.params)
        self.buckets = _bucket_list(cfg, self.layout.total)
        self._loss = float("nan")
        self._state = None            # carried hidden state (cfg.carry_hidden)
        self._err = 0                 # step error word (inject_error), max-reduced over ranks

    def reset_state(self) -> None:
        self._state = None

    def compute_params(self) -> Dict[str, torch.Tensor]:
        """The weights the step computes with: fp32 masters, or (bf16 working copies) the weight
        matrices rounded to bf16 -- from the gathered flat bf16 copy when the optimiser is sharded
        (other ranks' fp32 master slices are stale there) -- and the fp32 biases."""
        if not self.bf16:
            return self.params
        src = self.layout.views(self.flat_bf.float()) if self.flat_bf is not None else None
        return {k: (v if v.dim() == 1 else (src[k] if src is not None else v.to(torch.bfloat16).float()))
                for k, v in self.params.items()}

    def forward_backward(self, x: np.ndarray, y: np.ndarray) -> None:
        out = [] if self.cfg.carry_hidden else None
        loss, grads = cpu_ref.manual_backward(self.compute_params(), self.cfg, torch.from_numpy(np.asarray(x)),
                                              torch.from_numpy(np.asarray(y)), h0=self._state,
                                              state_out=out)
        if out is not None:
            self._state = out
        for k, g in grads.items():
            self.gviews[k].copy_(g)
        self._loss = float(loss)

    def inject_error(self, bits: int = 1) -> None:
        """Fault injection twin of Trainer::inject_error: this rank's step error word (sticky)."""
        self._err |= int(bits)

    def error_word(self) -> int:
        return self._err

    def _pipelined(self) -> bool:
        """CPU twin of Trainer::dp_pipe_on (one-layer data-parallel pipelined tail)."""
        c = self.cfg
        return (self.ctx.world > 1 and c.layers == 1 and self.shard is None and c.clip_norm <= 0
                and c.dp_pipeline == 1)

    def allreduce_grads(self) -> None:
        import torch.distributed as dist
        if self._pipelined():
            # twin of Trainer::record_dp_tail_l1: AR1 = [W_hh0 .. end) with the error word, then
            # AR2 = the FC pair (the device step all-reduces dP where this path has dW_ih0 / dEmb)
            r0 = self.layout["weight_hh_l0"].offset
            w1 = dist.all_reduce(self.flat_g[r0:], op=dist.ReduceOp.SUM, async_op=True)
            e = torch.tensor([self._err], dtype=torch.int64)
            dist.all_reduce(e, op=dist.ReduceOp.MAX)
            self._err = int(e.item())
            w2 = dist.all_reduce(self.flat_g[:r0], op=dist.ReduceOp.SUM, async_op=True)
            w1.wait()
            w2.wait()
            self.flat_g.div_(self.ctx.world)
            return
        allreduce_mean_buckets(self.flat_g, self.buckets, self.ctx.world)
        if self.ctx.world > 1:   # max over ranks, like the device word in the last collective
            e = torch.tensor([self._err], dtype=torch.int64)
            dist.all_reduce(e, op=dist.ReduceOp.MAX)
            self._err = int(e.item())

    def optimizer_step(self) -> None:
        if self._err:   # a step that failed on any rank is skipped on every rank
            return
        if self.shard is None and self._pipelined():   # Adam(all but FC), then Adam(FC), one step
            fc = ("fc.weight", "fc.bias")
            self.opt.step({k: v for k, v in self.params.items() if k not in fc},
                          {k: v for k, v in self.gviews.items() if k not in fc})
            self.opt.step({k: self.params[k] for k in fc}, {k: self.gviews[k] for k in fc}, advance=False)
            return
        if self.shard is None:
            self.opt.step(self.params, self.gviews)
            return
        import torch.distributed as dist
        c, sl = self.shard
        self.opt.step({k: self.flat_p[v] for k, v in sl.items()}, {k: self.flat_g[v] for k, v in sl.items()})
        if self.flat_bf is not None:
            # twin of record_sharded_opt mode 2: the owned slice's and the tail's bf16 copies, an
            # all-gather of the bf16 slices, and the owned fp32 biases as an integer-sum exchange
            W, r = self.ctx.world, self.ctx.rank
            self.flat_bf[sl["own"]] = self.flat_p[sl["own"]].to(torch.bfloat16)
            self.flat_bf[sl["tail"]] = self.flat_p[sl["tail"]].to(torch.bfloat16)
            if c:
                parts = list(self.flat_bf[:W * c].view(W, c).unbind(0))
                dist.all_gather(parts, self.flat_bf[sl["own"]].clone())
            idx = torch.cat([torch.arange(a, b) for a, b in self._bias_ranges])
            bits = self.flat_p[idx].view(torch.int32).clone()
            own = (idx >= r * c) & (idx < (r + 1) * c)
            pack = torch.where(own, bits, torch.zeros_like(bits))
            dist.all_reduce(pack, op=dist.ReduceOp.SUM)
            keep = idx < W * c
            self.flat_p[idx[keep]] = pack[keep].view(torch.float32)
            return
        if c:
            parts = list(self.flat_p[:self.ctx.world * c].view(self.ctx.world, c).unbind(0))
            dist.all_gather(parts, self.flat_p[sl["own"]].clone())

    def step(self, x, y) -> None:
        self.forward_backward(x, y)
        self.allreduce_grads()
        self.optimizer_step()

    def loss(self) -> float:
        return self._loss

    def gather_params(self) -> None:
        """Twin of Trainer::gather_params: with bf16 working copies gathered (shard_optim 2) the fp32
        master slices other ranks own are stale here until this all-gather."""
        if self.flat_bf is None or not self.shard[0]:
            return
        import torch.distributed as dist
        c, sl = self.shard
        parts = list(self.flat_p[:self.ctx.world * c].view(self.ctx.world, c).unbind(0))
        dist.all_gather(parts, self.flat_p[sl["own"]].clone())

    def state_dict(self) -> Dict[str, torch.Tensor]:
        self.gather_params()
        return {k: v.detach().clone() for k, v in self.params.items()}

    def grad_dict(self) -> Dict[str, torch.Tensor]:
        return {k: v.detach().clone() for k, v in self.gviews.items()}

    def opt_state(self):
        """(m, v, step): Adam moments as flat fp32 tensors in the flat layout.  COLLECTIVE when the
        optimiser is sharded -- every rank all-gathers the owned slices (the tail past world*c is
        identical everywhere), so all ranks must call it, not only the one that writes."""
        if self.shard is None:
            return to_flat(self.cfg, self.opt.m), to_flat(self.cfg, self.opt.v), self.opt.step_n
        import torch.distributed as dist
        c, sl = self.shard
        W, n = self.ctx.world, self.layout.total
        out = []
        for mom in (self.opt.m, self.opt.v):
            flat = torch.zeros(n, dtype=self.flat_p.dtype)
            if c:
                parts = list(flat[:W * c].view(W, c).unbind(0))
                dist.all_gather(parts, mom["own"].contiguous())
            flat[sl["tail"]] = mom["tail"]
            out.append(flat)
        return out[0], out[1], self.opt.step_n

    def load_opt_state(self, m: torch.Tensor, v: torch.Tensor, step: int) -> None:
        """Inverse of opt_state(): full flat moments in; a sharded rank keeps its own slices."""
        if self.shard is None:
            for dst, src in ((self.opt.m, m), (self.opt.v, v)):
                for k, x in from_flat(self.cfg, src.float()).items():
                    dst[k].copy_(x)
        else:
            _, sl = self.shard
            for dst, src in ((self.opt.m, m), (self.opt.v, v)):
                for k, s in sl.items():
                    dst[k].copy_(src[s])
        self.opt.step_n = int(step)


def make_trainer(cfg: GRUConfig, ctx: DistCtx, comm=None, params=None):
    if ctx.device.type == "cuda":
        return HipTrainer(cfg, ctx, params=params, comm=comm)
    return CpuTrainer(cfg, ctx, params=params)
