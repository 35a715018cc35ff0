"""Phase timing of the persistent forward sequence kernel (diagnostic stamps, 100 MHz clock).

Prints per-step durations of: wait (poll), A-load+MFMA+LDS partials, epilogue, publish.
"""
import os, sys, json, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from gru_mpi_cuda_amd.ops import load_ext

C = load_ext()
dev = torch.device("cuda", 0)
H, Bp, T, V = int(os.environ.get("H", 512)), int(os.environ.get("B", 256)), 32, 256
s = torch.cuda.current_stream().cuda_stream
HSb = torch.zeros(T + 1, Bp, H, device=dev, dtype=torch.bfloat16)
xch = torch.zeros(T, Bp, H, device=dev, dtype=torch.bfloat16)
HSf = torch.zeros(T + 1, Bp, H, device=dev)
HT = torch.zeros(H, (T + 1) * Bp, device=dev, dtype=torch.bfloat16)
sv = [torch.zeros(T, Bp, H, device=dev) for _ in range(4)]
Whh = (torch.randn(3 * H, H, device=dev) / H ** 0.5).bfloat16()
bhh = torch.zeros(3 * H, device=dev)
P = torch.randn(V, 3 * H, device=dev)
ids = torch.randint(0, V, (T, Bp), device=dev, dtype=torch.int32)
cnt = torch.zeros(Bp // 32 * H // 16 * 16 + 64, device=dev, dtype=torch.int32)
err = torch.zeros(16, device=dev, dtype=torch.int32)
dbg = torch.zeros(2 * 4096 * 8, device=dev, dtype=torch.int64)
d = dict(allow_local=int(os.environ.get("LOCAL", 1)), HSb=HSb.data_ptr(), xch=xch.data_ptr(), HSf=HSf.data_ptr(), HT=HT.data_ptr(), ldT=(T + 1) * Bp,
         sr=sv[0].data_ptr(), sz=sv[1].data_ptr(), sn=sv[2].data_ptr(), sghn=sv[3].data_ptr(),
         Whh=Whh.data_ptr(), bhh=bhh.data_ptr(), P=P.data_ptr(), ids=ids.data_ptr(),
         cnt=cnt.data_ptr(), err=err.data_ptr(), T=T, Bp=Bp, H=H,
         xring=int(os.environ.get("XR", 4)), tag=int(os.environ.get("TAG", 0)))
res = {}
for mode in ("plain", "dbg"):
    if mode == "dbg":
        d["dbg"] = dbg.data_ptr()
    times = []
    for it in range(20):
        cnt.zero_()
        xch.zero_()   # the tagged ring starts zeroed (in the engine: the backward zeroes it)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        C.fwd_seq(d, s)
        e1.record()
        torch.cuda.synchronize()
        times.append(e0.elapsed_time(e1) * 1000)
    res[mode + "_us"] = float(np.median(times[5:]))
res["err"] = int(err[0])
res["xring"], res["tag"] = d["xring"], d["tag"]
st = dbg.view(2, 4096, 8)[:, :T, :7].cpu().numpy().astype(np.float64) * 10.0   # ns
for wg in (0, 1):
    x = st[wg]
    ph = {"wait": x[1:, 1] - x[1:, 0], "mma": x[1:, 2] - x[1:, 1], "epi": x[1:, 3] - x[1:, 2],
          "pub": x[1:, 4] - x[1:, 3], "hsb": x[1:, 5] - x[1:, 4], "saves": x[1:, 6] - x[1:, 5],
          "loop": x[2:, 0] - x[1:-1, 6], "step": x[2:, 0] - x[1:-1, 0]}
    res[f"wg{wg}"] = {k: round(float(np.median(v)) / 1000, 3) for k, v in ph.items()}
print(json.dumps(res))
