import os, sys, json
sys.path.insert(0, "/root/repo")
import numpy as np, torch
from gru_mpi_cuda_amd.ops import load_ext
C = load_ext()
s = torch.cuda.current_stream().cuda_stream
C.spin_delay(0, s); torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    cs = torch.cuda.current_stream().cuda_stream
    for _ in range(20):
        C.spin_delay(0, cs)
ts = []
for it in range(10):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(); g.replay(); e1.record(); torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1) * 1000 / 20)
print(json.dumps({"trivial_us_per_launch": round(float(np.median(ts[3:])), 2)}))
