"""Placement census: which XCC ran each block of a grid (HW_REG_XCC_ID), for 256- and 512-thread
blocks at 256 and 1024 blocks, plus a persistent-kernel-sized grid run while another kernel
is resident."""
import os, sys, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from gru_mpi_cuda_amd.ops import load_ext
C = load_ext()
s = torch.cuda.current_stream().cuda_stream
res = {}
for nb, th in ((256, 512), (256, 256), (1024, 256)):
    seen = []
    for rep in range(5):
        out = torch.zeros(nb, dtype=torch.int32, device="cuda")
        C.xcc_census(out.data_ptr(), nb, th, s)
        torch.cuda.synchronize()
        v = out.cpu().tolist()
        rr = all(v[b] == v[b % 8] for b in range(nb))
        seen.append({"distinct": sorted(set(v)), "round_robin_mod8": rr, "first16": v[:16]})
    res[f"{nb}x{th}"] = seen
print(json.dumps(res))
