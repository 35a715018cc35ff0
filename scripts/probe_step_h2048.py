"""Time attribution of the large-H per-step kernels (gru_step_lds.hip) at H=2048, B=512: each kernel
launched back to back on fixed buffers, with and without its optional outputs, per variant.

    python scripts/probe_step_h2048.py  -> one JSON line per case (us per launch, mean of 200)
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gru_mpi_cuda_amd.ops import load_ext  # noqa: E402

H, B, T, V = 2048, 512, 4, 256
dev = "cuda"
C = load_ext()
g = torch.Generator(device=dev).manual_seed(0)


def rnd(*s, scale=1.0):
    return torch.randn(*s, device=dev, generator=g) * scale


def bf(t):
    return t.to(torch.bfloat16)


def timeit(fn, n=200):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1000 / n


s = torch.cuda.current_stream().cuda_stream
# ---- forward
hp = rnd(B, H, scale=0.5).clamp(-1, 1)
hpb, Whh, bhh = bf(hp), bf(rnd(3 * H, H, scale=H ** -0.5)), rnd(3 * H, scale=0.1)
P, ids = rnd(V, 3 * H), torch.randint(0, V, (B,), device=dev, dtype=torch.int32)
h_f, h_b = torch.empty(B, H, device=dev), torch.empty(B, H, device=dev, dtype=torch.bfloat16)
hT = torch.zeros(H, (T + 1) * B, device=dev, dtype=torch.bfloat16)
sv = [torch.empty(B, H, device=dev) for _ in range(4)]
base = dict(hprev_bf=hpb.data_ptr(), hprev_f=hp.data_ptr(), Whh=Whh.data_ptr(), bhh=bhh.data_ptr(), Bp=B, H=H,
            algo=2, P=P.data_ptr(), ids=ids.data_ptr(), h_f=h_f.data_ptr(), h_bf=h_b.data_ptr())
full = dict(base, hT=hT.data_ptr(), ldT=(T + 1) * B, colT=B, sr=sv[0].data_ptr(), sz=sv[1].data_ptr(),
            sn=sv[2].data_ptr(), sghn=sv[3].data_ptr())
for var in (dict(fwd8=2), dict(fwd8=1), dict(fwd8=0)):
    C.set_step_lds_variants(var)
    for tag, d in (("full", full), ("no_saves", dict(full, sr=0, sz=0, sn=0, sghn=0)),
                   ("no_saves_no_hT", base)):
        d = {k: v for k, v in d.items() if v != 0}
        print(json.dumps({"kernel": "fwd", "var": var, "case": tag, "us": round(timeit(lambda: C.fwd_step(d, s)), 2)}),
              flush=True)
C.set_step_lds_variants(dict(fwd8=2))
# ---- backward (split-K)
dgn = bf(rnd(B, 3 * H, scale=0.1))
WhhT = bf(rnd(H, 3 * H, scale=H ** -0.5))
carry, dy = rnd(B, H, scale=0.1), rnd(B, H, scale=0.1)
r, z, n = torch.sigmoid(rnd(B, H)), torch.sigmoid(rnd(B, H)), torch.tanh(rnd(B, H))
ghn, hpv = rnd(B, H), torch.tanh(rnd(B, H))
cout = torch.empty(B, H, device=dev)
dgh, dgi = (torch.empty(B, 3 * H, device=dev, dtype=torch.bfloat16) for _ in range(2))
dghT, dgiT = (torch.zeros(3 * H, T * B, device=dev, dtype=torch.bfloat16) for _ in range(2))
S_ = C.bwd_step_sk_splits(H, B)
part = torch.empty(H * B * S_, device=dev)
cnt = torch.zeros((H // 128) * (B // 128) * 16, device=dev, dtype=torch.int32)
err = torch.zeros(1, device=dev, dtype=torch.int32)
bb = dict(WhhT=WhhT.data_ptr(), dy=dy.data_ptr(), r=r.data_ptr(), z=z.data_ptr(), n=n.data_ptr(),
          ghn=ghn.data_ptr(), hprev=hpv.data_ptr(), carry_out=cout.data_ptr(), dgh=dgh.data_ptr(), Bp=B, H=H,
          algo=2, dgh_next=dgn.data_ptr(), carry_in=carry.data_ptr(), sk_part=part.data_ptr(),
          sk_part_floats=part.numel(), sk_cnt=cnt.data_ptr(), sk_cnt_words=cnt.numel(), err=err.data_ptr())
bfull = dict(bb, dghT=dghT.data_ptr(), dgiT=dgiT.data_ptr(), dgi=dgi.data_ptr(), ldT=T * B, colT=B)
for var in (dict(bwd_sk_pf=1), dict(bwd_sk_pf=0)):
    C.set_step_lds_variants(var)
    for tag, d in (("full", bfull), ("no_T_no_dgi", bb)):
        print(json.dumps({"kernel": "bwd_sk", "S": S_, "var": var, "case": tag,
                          "us": round(timeit(lambda: C.bwd_step(d, s)), 2)}), flush=True)
assert int(err.item()) == 0
