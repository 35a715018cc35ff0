#!/usr/bin/env python3
"""Headline benchmark (BASELINE.json): char-tokens/sec of a full GRU training step
(forward + softmax-xent + BPTT + gradient all-reduce + Adam), 1-layer GRU hidden=512,
256 sequences x 32 chars per GPU (weak scaling: global batch = 256 * N), bf16 MFMA compute
with fp32 master weights, synthetic name sequences, random-init weights.

    python bench.py --gpus N --steps K --warmup W
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

Without a launcher (no WORLD_SIZE in the environment) and --gpus N > 1, this process starts the N
rank processes itself (parallel/launch.py, one per GPU, 127.0.0.1 rendezvous) before anything
touches the GPU, and only relays their exit code; rank 0's JSON line is the output.  Under a
launcher, WORLD_SIZE must equal --gpus, and the RCCL communicator's own rank count
(ncclCommCount) is checked against it and reported as ``rccl_ranks``.

Rank 0 prints ONE JSON line; `value` is the whole-job aggregate (tokens/s over all ranks),
timed over exactly K steps bracketed by barrier + device synchronize, max over ranks.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

METRIC = "char-tokens/sec (whole node) for GRU hidden=512 at 1/2/4/8 MI355X"


def _launch_plan(K: int):
    """(G, lead) for K timed steps: `lead` single-step graph launches, then groups of G steps (G <= 32
    dividing K - lead).  Cost model from the headline's measurements: the first launch after the
    timed region's synchronize is the only one whose host work the GPU does not hide -- ~20 us for a
    single step, ~5 us per step + 40 us for a group (staging G batches, launching ~8G nodes,
    profiles/r3s5_host_group_launch.txt) -- and every graph boundary costs ~12.8 us
    (docs/DESIGN.md §6).  K = 20: 1 single + one group of 19; K = 300: 1 single + 13 groups of 23;
    K < 2: single steps only."""
    if K < 2:
        return 1, 0
    best = None
    for lead in range(0, min(8, K - 1) + 1):
        rest = K - lead
        for G in range(1, 33):
            if rest % G:
                continue
            launches = lead + rest // G
            first = 20.0 if lead else 5.0 * G + 40.0
            cost = first + 12.8 * (launches - 1)
            if best is None or cost < best[0] - 1e-9:
                best = (cost, G, lead)
    return best[1], best[2]


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--preset", default="h512")
    ap.add_argument("--per-gpu-batch", type=int, default=None,
                    help="override per-GPU batch (default: preset batch, 256 for h512)")
    ap.add_argument("--impl", choices=["hip", "torch"], default="hip",
                    help="hip = this engine; torch = torch.nn.GRU (MIOpen) comparator")
    ap.add_argument("--chunks", type=int, default=None)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--overlap", action="store_true",
                    help="chunked two-stream schedule instead of the persistent single-stream one")
    ap.add_argument("--rccl-self", action="store_true",
                    help="at 1 GPU, still record the gradient collectives (1-rank RCCL communicator) "
                         "to time the data-parallel step structure")
    ap.add_argument("--bucket-mb", type=float, default=None)
    ap.add_argument("--dp-pipeline", type=int, choices=[-1, 0, 1], default=None,
                    help="one-layer data-parallel tail: -1 auto (= one collective; the pipelined form measured "
                         "slower), 0 one collective, 1 pipelined")
    ap.add_argument("--shard-optim", type=int, nargs="?", const=1, default=-1, choices=[-1, 0, 1, 2],
                    help="sharded optimiser step (reduce-scatter, Adam on 1/world, all-gather of the fp32 "
                         "masters (1) or of the bf16 working copies (2)); -1 (default): the plan of "
                         "bench/cost_model.py for this preset and world size (1 GPU: replicated)")
    ap.add_argument("--min-warmup", type=int, default=300,
                    help="untimed steps before the timed region are at least this many: W from --warmup plus "
                         "max(0, N - W) extra, reported as extra_warmup_steps (a fresh box runs its first "
                         "~20 ms of steps below full clocks: W=5 measured 0.232-0.243 ms/step vs 0.221 after "
                         "100, profiles/r2_bench_warmup_probe.txt).  Same count on every rank.")
    ap.add_argument("--graph-steps", type=int, default=0,
                    help="hip engine on GPUs: G consecutive training steps captured into one graph launch "
                         "(1..32; the same G full steps, one graph boundary instead of G: ~13 us each at "
                         "the headline, docs/DESIGN.md §6); a remainder of K or W modulo G runs as "
                         "single-step graphs.  0 (default): a launch plan from the measured host / boundary "
                         "costs (_launch_plan: a few single-step launches first, so the first launch after "
                         "the timed region's synchronize is cheap, then groups).  Reported as graph_steps "
                         "and lead_single_steps.")
    ap.add_argument("--variant", action="append", default=[], metavar="KEY=INT",
                    help="kernel / step-plan variant (StepLdsVariants field, kernels.h; gemm.KEY: a GemmVariants "
                         "field), for A/B runs; repeatable")
    ap.add_argument("--launch-timeout", type=float, default=1800.0,
                    help="self-launch mode: wall-clock limit of the whole N-rank job in s")
    args = ap.parse_args()
    if args.steps < 1:
        ap.error("--steps must be >= 1")

    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        # no launcher: become the launcher (before any GPU call -- the parent never touches it)
        from gru_mpi_cuda_amd.parallel.launch import run
        return run(args.gpus, [os.path.abspath(__file__), *sys.argv[1:]], timeout=args.launch_timeout)
    if env_world is not None and int(env_world) != args.gpus and "--gpus" in " ".join(sys.argv):
        print(f"bench.py: WORLD_SIZE={env_world} but --gpus {args.gpus}", file=sys.stderr)
        return 2

    import torch
    import torch.distributed as dist
    from gru_mpi_cuda_amd.config import preset
    from gru_mpi_cuda_amd.parallel import dist as gdist
    from gru_mpi_cuda_amd.utils.data import NameStream

    ctx = gdist.init(use_gpu=torch.cuda.is_available())
    world = ctx.world
    if ctx.device.type == "cuda" and world > torch.cuda.device_count():
        print(f"bench.py: {world} ranks but only {torch.cuda.device_count()} visible GPUs", file=sys.stderr)
        return 2
    base = preset(args.preset)
    per_gpu = args.per_gpu_batch or base.batch
    cfg = base.replace(batch=per_gpu * world)
    if args.chunks:
        cfg = cfg.replace(time_chunks=args.chunks)
    if args.overlap:
        cfg = cfg.replace(overlap=True)
    if args.bucket_mb:
        cfg = cfg.replace(bucket_mb=args.bucket_mb)
    dp_plan = "replicated"
    if (args.shard_optim == -1 or args.dp_pipeline is None) and world > 1:
        # the world-aware plan from measured 1-GPU costs + the xGMI collective model
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "bench"))
        from cost_model import plan as _dp_plan
        dp_plan = _dp_plan(args.preset, world)
    shard = args.shard_optim if args.shard_optim != -1 else {"zero1_fp32": 1, "zero1_bf16": 2}.get(dp_plan, 0)
    if shard:
        cfg = cfg.replace(shard_optim=int(shard))
    if args.dp_pipeline is not None:
        cfg = cfg.replace(dp_pipeline=args.dp_pipeline)
    elif dp_plan == "pipelined":
        cfg = cfg.replace(dp_pipeline=1)

    stream = NameStream(per_gpu, cfg.seq, cfg.sos, cfg.eos, seed=1000 + ctx.rank, max_len=cfg.max_len)
    pool = [stream.next() for _ in range(8)]

    if args.impl == "hip":
        from gru_mpi_cuda_amd.engine.trainer import make_trainer
        if args.variant and ctx.device.type == "cuda":
            from gru_mpi_cuda_amd.ops import load_ext
            kv = [x.split("=", 1) for x in args.variant]   # "gemm.KEY=INT": a GemmVariants field
            step = {k: int(v) for k, v in kv if not k.startswith("gemm.")}
            gemm = {k[5:]: int(v) for k, v in kv if k.startswith("gemm.")}
            if step:
                load_ext().set_step_lds_variants(step)
            if gemm:
                load_ext().set_gemm_variants(gemm)
        from gru_mpi_cuda_amd.parallel.rccl import make_comm
        comm = make_comm(ctx) if ctx.device.type == "cuda" else None
        if comm is None and args.rccl_self and ctx.device.type == "cuda":
            from gru_mpi_cuda_amd.ops import load_ext
            C = load_ext()
            comm = C.RcclComm(C.RcclComm.unique_id(), 0, 1)
        if comm is not None and comm.count() != world:
            print(f"bench.py: RCCL communicator has {comm.count()} ranks, expected {world}", file=sys.stderr)
            return 2
        tr = make_trainer(cfg, ctx, comm=comm)
        if args.no_graph and hasattr(tr, "t"):
            tr.t.set_use_graph(False)
        step = lambda i: tr.step(*pool[i % len(pool)])  # noqa: E731
        G, lead = (args.graph_steps, 0) if args.graph_steps else _launch_plan(args.steps)
        if not (ctx.device.type == "cuda" and hasattr(tr, "steps")):
            G, lead = 1, 0
        final_loss = lambda: tr.loss()                  # noqa: E731
        plan = tr.t.plan() if hasattr(tr, "t") else "cpu"
    else:
        comm = None
        step, final_loss = _torch_gru_step(cfg, ctx, pool)
        plan = "torch.nn.GRU (MIOpen)"

    def sync():
        if ctx.device.type == "cuda":
            torch.cuda.synchronize(ctx.device)
        gdist.barrier()

    extra = max(0, args.min_warmup - args.warmup) if ctx.device.type == "cuda" else 0   # GPU clock ramp only
    if args.impl != "hip":
        G, lead = 1, 0
    single = step

    def run(i0, n):
        """n steps from pool index i0: `lead` single-step graphs, then whole groups of G steps per
        graph launch (the same steps, fewer graph boundaries), the remainder as single-step graphs"""
        i = 0
        for k in range(min(lead, n)):
            single(i0 + k)
            i += 1
        while G > 1 and i + G <= n:
            tr.steps([pool[(i0 + i + j) % len(pool)] for j in range(G)])
            i += G
        for k in range(i, n):
            single(i0 + k)

    run(0, args.warmup + extra)
    sync()
    t0 = time.perf_counter()
    run(args.warmup + extra, args.steps)
    sync()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=ctx.device if ctx.backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    loss = final_loss()
    if G > 1 and hasattr(tr, "t"):
        # what actually ran: steps() falls back to one graph per step (loudly) if a capture fails
        G = tr.t.graph_steps()
    tokens = cfg.batch * cfg.seq * args.steps
    value = tokens / el
    if ctx.is_main:
        out = {
            "metric": METRIC if args.preset in ("h512", "h512_dp8") else
                      f"char-tokens/sec (whole node) for GRU preset {args.preset}",
            "value": round(value, 1), "unit": "char-tokens/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "extra_warmup_steps": extra,
            "graph_steps": G, "lead_single_steps": lead,
            "ms_per_step": round(1000 * el / args.steps, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
            "data": "synthetic name sequences (seeded syllable generator), random-init weights",
            "config": {"model": f"GRU L={cfg.layers} H={cfg.hidden} E={cfg.embed} V={cfg.vocab}",
                       "global_batch": cfg.batch, "seq_len": cfg.seq,
                       "parallelism": f"dp{world}", "impl": args.impl,
                       "optimizer": cfg.optimizer, "time_chunks": cfg.time_chunks,
                       "overlap": cfg.overlap, "plan": plan, "shard_optim": int(cfg.shard_optim), "dp_plan": dp_plan,
                       "dp_pipeline": (int(tr.t.dp_tail_recorded()) if args.impl == "hip" and hasattr(tr, "t") else 0),
                       "collectives": (len(tr.t.allreduce_log()) if args.impl == "hip" and comm is not None
                                       and hasattr(tr, "t") else 0)},
            "rccl_ranks": comm.count() if comm is not None else (world if ctx.backend != "none" else 1),
            "comm_backend": "rccl" if comm is not None else ctx.backend,
            "final_loss": round(float(loss), 4),
        }
        print(json.dumps(out), flush=True)
    gdist.shutdown()
    return 0


def _torch_gru_step(cfg, ctx, pool):
    """torch.nn.GRU (MIOpen) comparator with the same model, loss and optimiser, bf16 autocast."""
    import torch
    import torch.nn as nn
    from torch.nn.parallel import DistributedDataParallel as DDP

    class Model(nn.Module):
        def __init__(self):
            super().__init__()
            self.emb = nn.Embedding(cfg.vocab, cfg.embed)
            self.gru = nn.GRU(cfg.embed, cfg.hidden, cfg.layers, batch_first=True)
            self.fc = nn.Linear(cfg.hidden, cfg.vocab)

        def forward(self, x):
            h, _ = self.gru(self.emb(x))
            return self.fc(h)

    dev = ctx.device
    m = Model().to(dev)
    model = DDP(m, device_ids=[dev.index]) if ctx.world > 1 else m
    opt = torch.optim.Adam(model.parameters(), lr=cfg.lr)
    dpool = [(torch.from_numpy(x).long().to(dev), torch.from_numpy(y).long().to(dev)) for x, y in pool]
    state = {"loss": None}

    def step(i):
        x, y = dpool[i % len(dpool)]
        with torch.autocast(device_type=dev.type, dtype=torch.bfloat16):
            logits = model(x)
            loss = nn.functional.cross_entropy(logits.float().reshape(-1, cfg.vocab), y.reshape(-1))
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()
        state["loss"] = loss.detach()

    return step, lambda: float(state["loss"])


if __name__ == "__main__":
    sys.exit(main())
