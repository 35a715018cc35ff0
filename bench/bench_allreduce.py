#!/usr/bin/env python3
"""Gradient-collective microbenchmark over the engine's own RCCL communicator (SURVEY §5.8:
"verify achieved bus BW in the bench"; the bucket-size choice of GRUConfig.bucket_mb).

For each message size it times `allreduce_avg_f32` on the native communicator (the call the
training step records into its graph) and torch.distributed's all_reduce for comparison, and
prints one JSON line per size with time, algorithm bandwidth (bytes / time) and bus bandwidth
(algbw * 2 (n-1) / n, the per-link figure that ring all-reduce is bound by on xGMI).

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 bench/bench_allreduce.py
    python bench/bench_allreduce.py            # 1 GPU: a 1-rank communicator (plumbing / launch cost)

The headline model's per-step gradient traffic is one ~5.25 MB collective (dP in the W_ih0 slot,
W_hh, biases, W_fc) after the backward.  `bench.py --dp-pipeline 1` records it instead as the
pipelined tail's two readiness buckets (Trainer::record_dp_tail_l1: AR1 = W_hh0, b_hh0, b_ih0, dP,
4.6 MB with the error word, beside the dW_fc K-slices; AR2 = the FC pair beside the embedding GEMMs
and the first Adam launch) -- measured slower on a 1-rank communicator (graph cross-stream edges,
profiles/r5_rccl_self_dp_pipeline1_timeline.txt), so it is opt-in.  The plan row below prints the
exact collectives of the captured step at this world size.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes-mb", default="0.25,1,2,4,5.25,8,16,32,64")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--no-plan", action="store_true",
                    help="skip the headline step's collective plan (the configuration the driver's N-GPU run records)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    from gru_mpi_cuda_amd.parallel import dist as gdist
    from gru_mpi_cuda_amd.parallel.rccl import make_comm
    from gru_mpi_cuda_amd.ops import load_ext

    ctx = gdist.init(use_gpu=True)
    C = load_ext()
    comm = make_comm(ctx) or C.RcclComm(C.RcclComm.unique_id(), 0, 1)
    dev = ctx.device
    stream = torch.cuda.current_stream(dev)
    n_ranks = ctx.world
    if not args.no_plan:
        _headline_plan(ctx, comm, stream, args)
    for mb in (float(x) for x in args.sizes_mb.split(",")):
        n = int(mb * (1 << 20) / 4) // 64 * 64
        buf = torch.ones(n, device=dev)

        def native():
            comm.allreduce_avg_f32(buf.data_ptr(), n, stream.cuda_stream)

        def via_torch():
            dist.all_reduce(buf)

        row = {"size_mb": round(n * 4 / 2 ** 20, 3), "ranks": n_ranks}
        for name, fn in (("native", native), ("torch", via_torch)):
            if name == "torch" and not dist.is_initialized():
                continue
            for _ in range(args.warmup):
                fn()
            torch.cuda.synchronize(dev)
            gdist.barrier()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(args.iters):
                fn()
            e1.record(stream)
            e1.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / args.iters
            algbw = n * 4 / (us * 1e-6) / 1e9
            busbw = algbw * (2 * (n_ranks - 1) / n_ranks if n_ranks > 1 else 1.0)
            row[name] = {"us": round(us, 2), "algbw_GBs": round(algbw, 1), "busbw_GBs": round(busbw, 1)}
        if ctx.is_main:
            print(json.dumps(row), flush=True)
    gdist.shutdown()
    return 0


def _headline_plan(ctx, comm, stream, args) -> None:
    """The exact collectives the headline step graph records at this world size (bench.py's config:
    preset h512, 256 sequences per GPU, default bucket_mb): Trainer::allreduce_log after one captured
    step -- (offset, floats) of each ncclAllReduce(avg), the last one grouped with the error-word max --
    and the same sizes replayed inside a captured hipGraph (how the step issues them), so the driver's
    first 8-GPU run has its collective cost measured in the form it will run."""
    import numpy as np
    import torch
    from gru_mpi_cuda_amd.config import preset
    from gru_mpi_cuda_amd.engine.trainer import make_trainer
    from gru_mpi_cuda_amd.utils.data import NameStream
    base = preset("h512")
    cfg = base.replace(batch=base.batch * ctx.world)
    tr = make_trainer(cfg, ctx, comm=comm)
    x, y = NameStream(base.batch, cfg.seq, seed=1000 + ctx.rank).next()
    tr.step(x, y)
    torch.cuda.synchronize(ctx.device)
    log = [(int(o), int(n)) for o, n in tr.t.allreduce_log()]
    buf = torch.ones(max([n for _, n in log] + [1]), device=ctx.device)
    g = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream(ctx.device)
    with torch.cuda.stream(side):
        with torch.cuda.graph(g, stream=side):
            for _, n in log:
                comm.allreduce_avg_f32(buf.data_ptr(), n, side.cuda_stream)
    for _ in range(args.warmup):
        g.replay()
    torch.cuda.synchronize(ctx.device)
    ts = []
    for _ in range(args.iters):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    if ctx.is_main:
        mb = sum(n for _, n in log) * 4 / 2 ** 20
        print(json.dumps({"headline_step_collectives": [{"offset": o, "floats": n, "mb": round(n * 4 / 2 ** 20, 3)}
                                                         for o, n in log],
                          "total_mb": round(mb, 3), "bucket_mb": cfg.bucket_mb, "ranks": ctx.world,
                          "plan": tr.t.plan(), "dp_pipeline": tr.t.dp_pipeline(),
                          "in_graph_replay_us_median": round(float(np.median(ts)), 2)}),
              flush=True)


if __name__ == "__main__":
    sys.exit(main())
