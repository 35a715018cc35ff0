"""Phase stamps of the forward with the FC pipeline (gru_fwd_seq_fc_kernel) vs the plain forward.
Per-step medians of: poll+loads (0->1), MFMA+partials (1->2), epilogue (2->3), publish drain (3->4),
row copy (4->5), rest (5->6), whole step."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from gru_mpi_cuda_amd.ops import load_ext
C = load_ext(build_if_missing=False)
dev = "cuda"
H, B, T, V = int(os.environ.get("H", 512)), int(os.environ.get("B", 256)), 32, 256
s = torch.cuda.current_stream().cuda_stream
bf = lambda t: t.to(torch.bfloat16).contiguous()
Whh = bf(torch.randn(3 * H, H, device=dev) / H ** 0.5)
Wfc = bf(torch.randn(V, H, device=dev) / H ** 0.5); WfcT = Wfc.t().contiguous()
bhh, bfc = torch.zeros(3 * H, device=dev), torch.zeros(V, device=dev)
P = torch.randn(V, 3 * H, device=dev)
ids = torch.randint(0, V, (T, B), device=dev, dtype=torch.int32)
labels = torch.randint(0, V, (T, B), device=dev, dtype=torch.int32)
inv = torch.full((1,), 1.0 / (T * B), device=dev)
HSb = torch.zeros(T + 1, B, H, device=dev, dtype=torch.bfloat16); xch = torch.zeros(T, B, H, device=dev, dtype=torch.bfloat16)
HSf = torch.zeros(T + 1, B, H, device=dev); HT = torch.zeros(H, (T + 1) * B, device=dev, dtype=torch.bfloat16)
HF = torch.zeros((T + 1) * B * H, device=dev, dtype=torch.bfloat16)
sv = [torch.zeros(T, B, H, device=dev) for _ in range(4)]
cnt = torch.zeros(B // 32 * H // 16 * 16 + 64, device=dev, dtype=torch.int32)
err = torch.zeros(16, device=dev, dtype=torch.int32)
dbg = torch.zeros(2 * 4096 * 8, device=dev, dtype=torch.int64)
xdl = torch.zeros(T * B * V, device=dev, dtype=torch.bfloat16); xdlT = torch.zeros_like(xdl)
xst = torch.zeros(T * (B // 32) * 16 * 64, device=dev)
dy = torch.zeros(T, B, H, device=dev); dW = torch.zeros(B // 32, V, H, device=dev); db = torch.zeros(B // 32, V, device=dev)
lp = torch.zeros(4096, device=dev)
d = dict(HSb=HSb.data_ptr(), xch=xch.data_ptr(), HSf=HSf.data_ptr(), HT=HT.data_ptr(), ldT=(T + 1) * B, HF=HF.data_ptr(),
         sr=sv[0].data_ptr(), sz=sv[1].data_ptr(), sn=sv[2].data_ptr(), sghn=sv[3].data_ptr(), Whh=Whh.data_ptr(),
         bhh=bhh.data_ptr(), P=P.data_ptr(), ids=ids.data_ptr(), cnt=cnt.data_ptr(), err=err.data_ptr(), T=T, Bp=B, H=H)
fd = dict(Wfc=Wfc.data_ptr(), WfcT=WfcT.data_ptr(), bfc=bfc.data_ptr(), labels=labels.data_ptr(), inv_count=inv.data_ptr(),
          xdl=xdl.data_ptr(), xdlT=xdlT.data_ptr(), xst=xst.data_ptr(), dy=dy.data_ptr(), dW_part=dW.data_ptr(),
          db_part=db.data_ptr(), loss_part=lp.data_ptr(), V=V)
for name in ("plain", "fc"):
    launch = (lambda: C.fwd_seq(d, s)) if name == "plain" else (lambda: C.fwd_seq_fc(d, fd, s))
    ts = []
    d.pop("dbg", None)
    for it in range(20):
        cnt.zero_()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); launch(); e1.record(); torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1000)
    d["dbg"] = dbg.data_ptr(); dbg.zero_(); cnt.zero_()
    launch(); torch.cuda.synchronize()
    st = dbg.view(2, 4096, 8).cpu().numpy().astype(np.int64)
    print(f"{name}: launch median {np.median(ts[3:]):.1f} us, err {int(err[0])}")
    nst = T + 3 if name == "fc" else T
    for wg in (0, 1):
        x = st[wg, :nst, :7].astype(np.float64) / 100.0
        ph = np.diff(x, axis=1)
        step = np.diff(x[:, 0])
        med = np.median(ph[2:T - 1], axis=0)
        print(f"  wg{wg}: per-step med {np.median(step[2:T - 1]):.3f} us | phases " + " ".join(f"{v:.3f}" for v in med)
              + f" | drain iters {[round(v, 2) for v in step[T - 1:]]}" if name == "fc" else
              f"  wg{wg}: per-step med {np.median(step[2:T - 1]):.3f} us | phases " + " ".join(f"{v:.3f}" for v in med))
