"""Standalone timing of the fused FC + softmax-xent (+ dH) kernel at the headline shape
(8192 tokens x V=256, H=512): python scripts/probe_fc.py  ->  one JSON line."""
import os, sys, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from gru_mpi_cuda_amd.ops import load_ext

C = load_ext()
if "FLASH" in os.environ:   # StepLdsVariants.fc_flash: 1 fc_xent_fl, 0 the two-stream 8-wave kernel
    C.set_step_lds_variants(dict(fc_flash=int(os.environ["FLASH"])))
dev = torch.device("cuda", 0)
M, H, V = int(os.environ.get("M", 8192)), int(os.environ.get("H", 512)), 256
s = torch.cuda.current_stream().cuda_stream
X = (torch.randn(M, H, device=dev)).bfloat16()
W = (torch.randn(V, H, device=dev) / H ** 0.5).bfloat16()
WT = W.T.contiguous()
from gru_mpi_cuda_amd.ops import ft_layout
Wf, WTf = ft_layout(W), ft_layout(WT)
b = torch.randn(V, device=dev) * 0.1
y = torch.randint(0, V, (M,), device=dev, dtype=torch.int32)
inv = torch.tensor([1.0 / M], device=dev)
dlT = torch.empty(V, M, device=dev, dtype=torch.bfloat16)
lp = torch.empty(M // 32, device=dev)
dy = torch.empty(M, H, device=dev)
d = dict(X=X.data_ptr(), W=W.data_ptr(), b=b.data_ptr(), labels=y.data_ptr(), inv_count=inv.data_ptr(),
         dlT=dlT.data_ptr(), loss_part=lp.data_ptr(), M=M, H=H, V=V, ldT=M, colT=0,
         WT=WT.data_ptr(), dy=dy.data_ptr(), Wf=Wf.data_ptr(), WTf=WTf.data_ptr())
# 20 launches captured in one graph: host launch overhead out of the measurement
C.fc_xent(d, s)
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    cs = torch.cuda.current_stream().cuda_stream
    for _ in range(20):
        C.fc_xent(d, cs)
times = []
for it in range(10):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    times.append(e0.elapsed_time(e1) * 1000 / 20)
logits = X.float() @ W.float().T + b
ref_loss = torch.nn.functional.cross_entropy(logits, y.long()).item()
p = torch.softmax(logits, -1)
p[torch.arange(M), y.long()] -= 1
ref_dy = (p / M) @ W.float()
err = (dy - ref_dy).abs().max().item()
dbg = torch.zeros(32, device=dev, dtype=torch.int64)
d["dbg"] = dbg.data_ptr()
C.fc_xent(d, s)
torch.cuda.synchronize()
st = dbg.cpu().numpy().astype(np.float64)
waves = st[16:24]
st = st[:16]
n = int((st > 0).sum())
if waves.min() > 0:   # per-wave "logits done" relative to wave 0's stamp at the start
    print(json.dumps({"logits_done_us_per_wave": [round((x - st[0]) * 0.01, 2) for x in waves]}))
phases = [round((st[i + 1] - st[i]) * 0.01, 2) for i in range(n - 1)]   # 100 MHz -> us
print(json.dumps({"phases_us_wg0": phases}))
print(json.dumps({"M": M, "H": H, "V": V, "us": round(float(np.median(times[5:])), 2),
                  "loss_err": abs(lp.sum().item() - ref_loss), "dy_err": err}))
