"""Phase timing of the one-layer forward with the FC head inside (gru_fwd_seq_fc) at the headline shape.

Times (median of 20 launches, events) the plain persistent forward and the FC-consumer launch in
four probe modes -- consumers that leave at once (the census then covers the producers only: the
cost of the 128-VGPR build alone), that stop after the placement census (+ waiting for the consumers'
dispatch), after their FC items, and the full kernel (+8: the recurrence at s_setprio 2; +16: the
FC build without the 128-VGPR cap, with mode 3 only; mode 4: the items without their W_fc / W_fc^T
fragment loads) -- and reads the 100 MHz
phase stamps of workgroup 0 (a recurrence block) and of the last workgroup (the consumer of row
block 7's step 31: the item on the critical path).
"""
import os, sys, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from gru_mpi_cuda_amd.ops import load_ext

C = load_ext()
dev = torch.device("cuda", 0)
H, Bp, T, V = 512, int(os.environ.get("B", 256)), 32, 256
s = torch.cuda.current_stream().cuda_stream
bf = torch.bfloat16
HSb = torch.zeros(T + 1, Bp, H, device=dev, dtype=bf)
xch = torch.zeros(T, Bp, H, device=dev, dtype=bf)
HSf = torch.zeros(T + 1, Bp, H, device=dev)
HF = torch.zeros(T + 1, Bp, H, device=dev, dtype=bf)
sv = [torch.zeros(T, Bp, H, device=dev) for _ in range(4)]
Whh = (torch.randn(3 * H, H, device=dev) / H ** 0.5).to(bf)
bhh = torch.zeros(3 * H, device=dev)
P = torch.randn(V, 3 * H, device=dev)
ids = torch.randint(0, V, (T, Bp), device=dev, dtype=torch.int32)
cnt = torch.zeros(Bp // 32 * (H // 16 + 32) * 16 + 64, device=dev, dtype=torch.int32)
err = torch.zeros(16, device=dev, dtype=torch.int32)
dbg = torch.zeros(2 * 4096 * 8, device=dev, dtype=torch.int64)
Wf = (torch.randn(V * H, device=dev) / H ** 0.5).to(bf)
WTf = (torch.randn(V * H, device=dev) / V ** 0.5).to(bf)
bfc = torch.zeros(V, device=dev)
labels = torch.randint(0, V, (T, Bp), device=dev, dtype=torch.int32)
inv = torch.full((1,), 1.0 / (T * Bp), device=dev)
dy = torch.zeros(T * Bp, H, device=dev)
dlF = torch.zeros(T * Bp * V, device=dev, dtype=bf)
loss = torch.zeros(T * Bp // 32, device=dev)
dW = torch.zeros(Bp // 32, V, H, device=dev)
db = torch.zeros(Bp // 32, V, device=dev)
d = dict(allow_local=int(os.environ.get("LOCAL", 1)), HSb=HSb.data_ptr(), xch=xch.data_ptr(), HSf=HSf.data_ptr(),
         HF=HF.data_ptr(), sr=sv[0].data_ptr(), sz=sv[1].data_ptr(), sn=sv[2].data_ptr(), sghn=sv[3].data_ptr(),
         Whh=Whh.data_ptr(), bhh=bhh.data_ptr(), P=P.data_ptr(), ids=ids.data_ptr(),
         cnt=cnt.data_ptr(), err=err.data_ptr(), T=T, Bp=Bp, H=H, xring=4)
fd = dict(Wf=Wf.data_ptr(), WTf=WTf.data_ptr(), b=bfc.data_ptr(), labels=labels.data_ptr(), inv_count=inv.data_ptr(),
          dy=dy.data_ptr(), dlF=dlF.data_ptr(), loss_part=loss.data_ptr(), dW=dW.data_ptr(), db=db.data_ptr(), V=V)


def run(fn, n=20):
    times = []
    for _ in range(n):
        cnt.zero_()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        times.append(e0.elapsed_time(e1) * 1000)
    return round(float(np.median(times[5:])), 2)


res = {"fc_supported": bool(C.fwd_seq_fc_supported(H, Bp, V))}
res["plain_us"] = run(lambda: C.fwd_seq(d, s))
for probe in [int(x) for x in os.environ.get("PROBES", "3,19,1,2,4,0,10,8").split(",")]:
    fd["probe"] = probe
    res[f"fc_probe{probe}_us"] = run(lambda: C.fwd_seq_fc(d, fd, s))
res["err"] = int(err[0])
# stamps of the full kernel
d["dbg"] = dbg.data_ptr()
fd["probe"] = 0
for name, fn in (("plain", lambda: C.fwd_seq(d, s)), ("fc", lambda: C.fwd_seq_fc(d, fd, s))):
    dbg.zero_()
    run(fn, n=3)
    st = dbg.view(2, 4096, 8).cpu().numpy().astype(np.float64) * 10.0 / 1000.0   # us
    x = st[0, :T, :7]
    step = np.diff(x[:, 0])
    out = {"rec_step_us_median": round(float(np.median(step[1:])), 3),
           "rec_first_to_last_step_us": round(float(x[T - 1, 6] - x[0, 0]), 2)}
    if name == "fc":
        c = st[1, T - 1, :4]   # last consumer's item (step 31): after wait / X tile / softmax / done
        out["last_item_wait_end_rel_rec_end_us"] = round(float(c[0] - x[T - 1, 6]), 3)
        out["last_item_xtile_us"] = round(float(c[1] - c[0]), 3)
        out["last_item_logits_softmax_us"] = round(float(c[2] - c[1]), 3)
        out["last_item_dh_done_us"] = round(float(c[3] - c[2]), 3)
    res[name] = out
print(json.dumps(res))
