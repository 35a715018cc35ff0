"""Host-side cost of one multi-step graph launch at the headline (the part of the bench's timed region
the GPU does not hide on the first launch after a sync): set_batches for G batches, step_group."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from gru_mpi_cuda_amd.config import preset
from gru_mpi_cuda_amd.engine.trainer import HipTrainer
from gru_mpi_cuda_amd.utils.data import NameStream
cfg = preset("h512")
tr = HipTrainer(cfg)
ds = NameStream(cfg.batch, cfg.seq, seed=1)
pool = [ds.next() for _ in range(32)]
for G in (4, 10):
    for _ in range(3):
        tr.steps(pool[:G])
    torch.cuda.synchronize()
    ts, tl, tw = [], [], []
    for it in range(10):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        xs = np.stack([np.asarray(x) for x, _ in pool[:G]]); ys = np.stack([np.asarray(y) for _, y in pool[:G]])
        tr.t.set_batches(xs, ys)
        t1 = time.perf_counter()
        tr.t.step_group(tr._stream())
        t2 = time.perf_counter()
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        ts.append((t1 - t0) * 1e6); tl.append((t2 - t1) * 1e6); tw.append((t3 - t0) * 1e6)
    print(f"G={G}: set_batches {np.median(ts):.1f} us, step_group launch {np.median(tl):.1f} us, "
          f"sync-to-sync {np.median(tw):.1f} us ({np.median(tw) / G:.1f} per step)")
