"""Diagnostic: table-free forward vs the P-table forward (small-GEMM table and torch table)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from gru_mpi_cuda_amd.ops import load_ext
ext = load_ext(build_if_missing=False)
DEV = "cuda"
S = lambda: torch.cuda.current_stream().cuda_stream
bf = lambda t: t.to(torch.bfloat16).contiguous()
H, B, T, V, E = 512, 256, 8, 256, 512
g = torch.Generator(device="cpu").manual_seed(11)
R = lambda *s, sc=1.0: (torch.randn(*s, generator=g) * sc).to(DEV)
Whh, Wih = bf(R(3 * H, H, sc=H ** -0.5)), bf(R(3 * H, E, sc=E ** -0.5))
Emb, bhh, bih = bf(R(V, E, sc=0.7)), R(3 * H, sc=0.1), R(3 * H, sc=0.1)
ids = torch.randint(0, V, (T, B), generator=g, dtype=torch.int32).to(DEV)
P = torch.full((V, 3 * H), float("nan"), device=DEV)
ext.gemm_nt(dict(A=Emb.data_ptr(), lda=E, B=Wih.data_ptr(), ldb=E, C=P.data_ptr(), ldc=3 * H, M=V, N=3 * H, K=E,
                 splits=1, algo=3, bias=bih.data_ptr()), S())
Pr = Emb.float() @ Wih.float().t() + bih
torch.cuda.synchronize()
print("P small-gemm vs torch max", (P - Pr).abs().max().item())
slot = torch.zeros(16 + 2 * B * T, dtype=torch.int32)
slot[0] = B
slot[1] = torch.tensor([0.5], dtype=torch.float32).view(torch.int32)
slot[16:16 + B * T] = ids.t().contiguous().flatten().cpu()
slot[16 + B * T:] = 3
slot = slot.to(DEV)
def run(mode, table=None, prep=False, fill=None):
    err = torch.zeros(16, device=DEV, dtype=torch.int32)
    HSb = torch.zeros(T + 1, B, H, device=DEV, dtype=torch.bfloat16)
    xch = torch.zeros(T, B, H, device=DEV, dtype=torch.bfloat16)
    HSf = torch.zeros(T + 1, B, H, device=DEV)
    sv = [torch.zeros(T, B, H, device=DEV) for _ in range(4)]
    cnt = torch.zeros(B // 32 * H // 16 * 16 + 64, device=DEV, dtype=torch.int32)
    idb = ids.clone() if fill is None else torch.full_like(ids, fill)
    lab = torch.zeros_like(ids); inv = torch.zeros(1, device=DEV)
    d = dict(HSb=HSb.data_ptr(), xch=xch.data_ptr(), HSf=HSf.data_ptr(), sr=sv[0].data_ptr(), sz=sv[1].data_ptr(),
             sn=sv[2].data_ptr(), sghn=sv[3].data_ptr(), Whh=Whh.data_ptr(), bhh=bhh.data_ptr(), cnt=cnt.data_ptr(),
             err=err.data_ptr(), ids=idb.data_ptr(), T=T, Bp=B, H=H)
    if mode == "pl":
        d.update(Emb=Emb.data_ptr(), Wih0=Wih.data_ptr(), bih=bih.data_ptr(), V=V, E=E)
        if prep:
            d.update(prep_in=slot.data_ptr(), Bmax=B, labels=lab.data_ptr(), inv_count=inv.data_ptr())
    else:
        d.update(P=table.data_ptr())
    ext.fwd_seq(d, S())
    torch.cuda.synchronize()
    print(mode, prep, fill, "err", int(err[0]), "ids ok", torch.equal(idb, ids))
    return HSf, sv
h_pl, sv_pl = run("pl")
h_sg, sv_sg = run("tab", P)
h_tr, sv_tr = run("tab", Pr.contiguous())
# step 0 gates isolate gi: r = sigmoid(gi_r + bhh_r) at t=0 (h = 0)
for name, (h, sv) in {"small": (h_sg, sv_sg), "torch": (h_tr, sv_tr)}.items():
    print(name, "HSf max diff vs pl", (h - h_pl).abs().max().item(), "r0 max diff", (sv[0][0] - sv_pl[0][0]).abs().max().item())
gi_pl = torch.logit(sv_pl[0][0].double()) - bhh[:H].double()
gi_ref = P[ids[0].long()][:, :H].double()
dd = (gi_pl - gi_ref).abs()
print("gi_r from pl r-gate vs table: max", dd.max().item())
idx = (dd > 1e-3).nonzero()
print("bad entries", idx.shape[0], idx[:10].tolist())

for fill in (None, -7, 5):
    h_p, _ = run("pl", prep=True, fill=fill)
    dd = (h_p - h_sg).abs().amax(dim=2)   # [T+1][B]
    bad = (dd > 0).nonzero()
    print("prep fill", fill, "max", dd.max().item(), "bad (t,b) count", bad.shape[0], "rows", sorted(set(bad[:, 1].tolist()))[:40], "first t", bad[:, 0].min().item() if bad.shape[0] else None)
