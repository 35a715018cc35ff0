"""Table-free layer-0 forward (PL) vs the table forward: launch times and prologue / step stamps.
modes: table | pl (ids given) | pl+prep device slot | pl+prep pinned host slot"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from gru_mpi_cuda_amd.ops import load_ext
C = load_ext(build_if_missing=False)
dev = "cuda"
H, B, T, V, E = 512, 256, 32, 256, 512
s = torch.cuda.current_stream().cuda_stream
bf = lambda t: t.to(torch.bfloat16).contiguous()
Whh, Wih, Emb = bf(torch.randn(3 * H, H, device=dev) / H ** 0.5), bf(torch.randn(3 * H, E, device=dev) / E ** 0.5), bf(torch.randn(V, E, device=dev))
bhh, bih = torch.zeros(3 * H, device=dev), torch.zeros(3 * H, device=dev)
P = torch.randn(V, 3 * H, device=dev)
ids = torch.randint(0, V, (T, B), device=dev, dtype=torch.int32)
slot_d = torch.zeros(16 + 2 * B * T, dtype=torch.int32); slot_d[0] = B
slot_d[16:16 + B * T] = ids.t().contiguous().flatten().cpu()
slot_h = slot_d.pin_memory(); slot_d = slot_d.to(dev)
lab = torch.zeros(T, B, device=dev, dtype=torch.int32); inv = torch.zeros(1, device=dev)
HSb = torch.zeros(T + 1, B, H, device=dev, dtype=torch.bfloat16); xch = torch.zeros(T, B, H, device=dev, dtype=torch.bfloat16)
HSf = torch.zeros(T + 1, B, H, device=dev); HT = torch.zeros(H, (T + 1) * B, device=dev, dtype=torch.bfloat16)
sv = [torch.zeros(T, B, H, device=dev) for _ in range(4)]
cnt = torch.zeros(B // 32 * H // 16 * 16 + 64, device=dev, dtype=torch.int32)
err = torch.zeros(16, device=dev, dtype=torch.int32)
dbg = torch.zeros(2 * 4096 * 8, device=dev, dtype=torch.int64)
base = dict(HSb=HSb.data_ptr(), xch=xch.data_ptr(), HSf=HSf.data_ptr(), HT=HT.data_ptr(), ldT=(T + 1) * B,
            sr=sv[0].data_ptr(), sz=sv[1].data_ptr(), sn=sv[2].data_ptr(), sghn=sv[3].data_ptr(), Whh=Whh.data_ptr(),
            bhh=bhh.data_ptr(), ids=ids.data_ptr(), cnt=cnt.data_ptr(), err=err.data_ptr(), T=T, Bp=B, H=H)
pl = dict(Emb=Emb.data_ptr(), Wih0=Wih.data_ptr(), bih=bih.data_ptr(), V=V, E=E)
modes = {"table": dict(P=P.data_ptr()), "pl": pl,
         "pl+prep_dev": dict(pl, prep_in=slot_d.data_ptr(), Bmax=B, labels=lab.data_ptr(), inv_count=inv.data_ptr()),
         "pl+prep_host": dict(pl, prep_in=slot_h.data_ptr(), Bmax=B, labels=lab.data_ptr(), inv_count=inv.data_ptr())}
for name, extra in modes.items():
    d = dict(base, **extra)
    ts = []
    for it in range(30):
        cnt.zero_()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); C.fwd_seq(d, s); e1.record(); torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1000)
    d["dbg"] = dbg.data_ptr(); dbg.zero_(); cnt.zero_()
    C.fwd_seq(d, s); torch.cuda.synchronize()
    st = dbg.view(2, 4096, 8).cpu().numpy().astype(np.int64)
    out = [f"{name:13s} launch med {np.median(ts[5:]):6.1f} us (err {int(err[0])})"]
    for wg in (0, 1):
        pro = st[wg, T + 1, :5]
        t0 = pro[0]
        loop0 = st[wg, 0, 0]
        end = st[wg, T - 1, 6]
        rel = lambda v: (v - t0) / 100.0 if v else float('nan')
        out.append(f"  wg{wg}: prologue stamps {[round(rel(v), 2) for v in pro]} loop start {rel(loop0):.2f} end {rel(end):.2f} "
                   f"per-step {(end - loop0) / 100.0 / T:.3f}")
    print("\n".join(out))
