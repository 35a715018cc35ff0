"""Where the fixed cost of bench.py's timed region goes (driver form: K = 20 steps, 1 single-step graph
+ one 19-step graph): host stamps after each call, GPU events around the region and around each
launch, against the same K steps' kernel time.  One JSON line per configuration.
    python scripts/probe_launch_overhead.py"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from gru_mpi_cuda_amd.config import preset
from gru_mpi_cuda_amd.engine.trainer import HipTrainer
from gru_mpi_cuda_amd.utils.data import NameStream

cfg = preset("h512")
tr = HipTrainer(cfg)
stream = NameStream(cfg.batch, cfg.seq, cfg.sos, cfg.eos, seed=1000, max_len=cfg.max_len)
pool = [stream.next() for _ in range(8)]


def run(i0, n, lead, G):
    i = 0
    for k in range(min(lead, n)):
        tr.step(*pool[(i0 + k) % 8])
        i += 1
    while G > 1 and i + G <= n:
        tr.steps([pool[(i0 + i + j) % 8] for j in range(G)])
        i += G
    for k in range(i, n):
        tr.step(*pool[(i0 + k) % 8])


import numpy as np


def parts(G):
    """host time of the pieces of one group launch: numpy stack, staging (C++ fill + H2D), graph launch"""
    bs = [pool[j % 8] for j in range(G)]
    if tr.t.graph_steps() != G:
        tr.t.set_graph_steps(G)
    s = torch.cuda.current_stream().cuda_stream
    t0 = time.perf_counter()
    xs = np.stack([np.asarray(x) for x, _ in bs]); ys = np.stack([np.asarray(y) for _, y in bs])
    t1 = time.perf_counter()
    tr.t.set_batches(xs, ys)
    t2 = time.perf_counter()
    tr.t.step_group(s)
    t3 = time.perf_counter()
    torch.cuda.synchronize()
    return {"stack_us": round((t1 - t0) * 1e6, 1), "stage_us": round((t2 - t1) * 1e6, 1),
            "launch_us": round((t3 - t2) * 1e6, 1)}


for lead, G in ((1, 19), (2, 18), (3, 17), (1, 19), (2, 18), (3, 17)):
    run(0, 300, 1, 23)   # warm: clocks up
    run(0, 20, lead, G)  # both graphs of this plan captured
    torch.cuda.synchronize()
    pr = [parts(G) for _ in range(3)][-1]
    single = []
    for _ in range(3):
        t0 = time.perf_counter()
        tr.step(*pool[0])
        single.append(round((time.perf_counter() - t0) * 1e6, 1))
        torch.cuda.synchronize()
    run(0, 20, lead, G)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    t0 = time.perf_counter()
    ev[0].record()
    h = []
    for k in range(lead):
        tr.step(*pool[k % 8])
        h.append(time.perf_counter() - t0)
    ev[1].record()
    tr.steps([pool[(lead + j) % 8] for j in range(G)])
    h.append(time.perf_counter() - t0)
    ev[2].record()
    torch.cuda.synchronize()
    t_end = time.perf_counter() - t0
    print(json.dumps({"lead": lead, "G": G, "host_elapsed_us": round(t_end * 1e6, 1),
                      "host_stamps_us": [round(x * 1e6, 1) for x in h],
                      "gpu_region_us": round(ev[0].elapsed_time(ev[2]) * 1e3, 1),
                      "single_host_us": single, "group_parts": pr,
                      "ms_per_step_host": round(t_end * 1e3 / (lead + G), 4)}), flush=True)
