"""Timeline of the fused step tail (tail.hip) at the headline: per-item s_memrealtime stamps
(start, wait done, end) of the last step, summarised per item kind.  usage: probe_tail.py [steps]"""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from gru_mpi_cuda_amd.config import preset
from gru_mpi_cuda_amd.engine.trainer import HipTrainer
from gru_mpi_cuda_amd.utils.data import NameStream

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
cfg = preset("h512")
tr = HipTrainer(cfg)
dbg = torch.zeros(65536 * 4, dtype=torch.int64, device="cuda")
tr.t.set_tail_dbg(dbg.data_ptr())
ds = NameStream(cfg.batch, cfg.seq, seed=1)
for _ in range(steps):
    tr.step(*ds.next())
torch.cuda.synchronize()
plan = tr.t.tail_plan()
names = ["prep", "dWfc", "dP", "loss", "adam", "dWih0", "dEmb", "P"]
n = sum(plan)
d = dbg[: 4 * n].view(n, 4).cpu().numpy().astype(np.int64)
t0 = d[:, 0].min()
st, wt, en = (d[:, 0] - t0) / 100.0, (d[:, 1] - t0) / 100.0, (d[:, 2] - t0) / 100.0   # us (100 MHz)
print(f"plan {dict(zip(names, plan))} items {n}, span {en.max():.2f} us, wgs {len(set(d[:, 3] & 0xffff))}")
o = 0
for name, c in zip(names, plan):
    if c:
        s, w, e = st[o:o + c], wt[o:o + c], en[o:o + c]
        waited = d[o:o + c, 1] > 0
        wdur = np.where(waited, w - s, 0.0)
        print(f"{name:6s} n={c:4d} start[{s.min():6.2f},{np.median(s):6.2f},{s.max():6.2f}] "
              f"end[{e.min():6.2f},{np.median(e):6.2f},{e.max():6.2f}] dur med {np.median(e - s):5.2f} max {np.max(e - s):5.2f} "
              f"wait med {np.median(wdur):5.2f} max {np.max(wdur):5.2f}")
    o += c
