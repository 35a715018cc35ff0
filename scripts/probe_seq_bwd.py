"""Phase timing of the persistent backward sequence kernel (fused dW_hh + dP), 100 MHz stamps."""
import os, sys, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from gru_mpi_cuda_amd.ops import load_ext

C = load_ext()
dev = torch.device("cuda", 0)
H, Bp, T, V = int(os.environ.get("H", 512)), int(os.environ.get("B", 256)), int(os.environ.get("T", 32)), 256
R16 = int(os.environ.get("R16", 0))     # 1: the 16-row-block kernel (gru_seq16.hip)
H3, nrb = 3 * H, Bp // (16 if R16 else 32)
fuse_w, fuse_p = int(os.environ.get("FW", 1)), int(os.environ.get("FP", 1))
s = torch.cuda.current_stream().cuda_stream
f = lambda *sh: torch.randn(*sh, device=dev) * 0.1          # noqa: E731
dy, sr, sz, sn, sghn = f(T, Bp, H), torch.rand(T, Bp, H, device=dev), torch.rand(T, Bp, H, device=dev), \
    torch.tanh(f(T, Bp, H)), f(T, Bp, H)
HSf = f(T + 1, Bp, H)
HT = f(H, (T + 1) * Bp).bfloat16()
HF = f((T + 1) * Bp * H).bfloat16()     # fragment-tiled h (SeqBwdArgs::HF); values irrelevant here
WhhT = (torch.randn(H, H3, device=dev) / H ** 0.5).bfloat16()
xbuf = torch.zeros(T, Bp, H3, device=dev, dtype=torch.bfloat16)
dghT = torch.zeros(H3, T * Bp, device=dev, dtype=torch.bfloat16)
dgiT = torch.zeros_like(dghT)
dWp = torch.zeros(nrb, H3, H, device=dev)
dbh, dbi = torch.zeros(nrb, H3, device=dev), torch.zeros(nrb, H3, device=dev)
ids = torch.randint(0, V, (T, Bp), device=dev, dtype=torch.int32)
dPp = torch.zeros(nrb, V, H3, device=dev)
cnt = torch.zeros(nrb * H // 16 * 16 + 64, device=dev, dtype=torch.int32)
err = torch.zeros(16, device=dev, dtype=torch.int32)
dbg = torch.zeros(2 * 4096 * 8, device=dev, dtype=torch.int64)
d = dict(allow_local=int(os.environ.get("LOCAL", 1)), dy=dy.data_ptr(), sr=sr.data_ptr(), sz=sz.data_ptr(), sn=sn.data_ptr(), sghn=sghn.data_ptr(),
         HSf=HSf.data_ptr(), HT=HT.data_ptr(), ldT=(T + 1) * Bp, WhhT=WhhT.data_ptr(), xbuf=xbuf.data_ptr(),
         dbhh_part=dbh.data_ptr(), dbih_part=dbi.data_ptr(), cnt=cnt.data_ptr(), err=err.data_ptr(),
         T=T, Bp=Bp, H=H, V=V, rows16=R16, xring=int(os.environ.get("XR", 0)))
if fuse_w:
    d["dWhh_part"] = dWp.data_ptr()
    if int(os.environ.get("HF", 1)):
        d["HF"] = HF.data_ptr()
if fuse_p:
    d.update(ids=ids.data_ptr(), dP_part=dPp.data_ptr())
if not (fuse_w and fuse_p):
    d.update(dghT=dghT.data_ptr(), dgiT=dgiT.data_ptr(), ldG=T * Bp)
res = {"H": H, "Bp": Bp, "T": T, "fuse_w": fuse_w, "fuse_p": fuse_p, "rows16": R16, "xring": int(os.environ.get("XR", 0))}
for mode in ("plain", "dbg"):
    if mode == "dbg":
        d["dbg"] = dbg.data_ptr()
    times = []
    for it in range(20):
        cnt.zero_()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        C.bwd_seq(d, s)
        e1.record()
        torch.cuda.synchronize()
        times.append(e0.elapsed_time(e1) * 1000)
    res[mode + "_us"] = round(float(np.median(times[5:])), 1)
res["err"] = int(err[0])
st = dbg.view(2, 4096, 8)[:, :T, :7].cpu().numpy().astype(np.float64) * 10.0
for wg in (0, 1):
    x = st[wg]
    ph = {"wait": x[1:, 1] - x[1:, 0], "mma": x[1:, 2] - x[1:, 1], "epi": x[1:, 3] - x[1:, 2],
          "pub": x[1:, 4] - x[1:, 3], "dgi": x[1:, 5] - x[1:, 4], "fused": x[1:, 6] - x[1:, 5],
          "loop": x[2:, 0] - x[1:-1, 6], "step": x[2:, 0] - x[1:-1, 0]}
    res[f"wg{wg}"] = {k: round(float(np.median(v)) / 1000, 3) for k, v in ph.items()}
print(json.dumps(res))
