"""Standalone timing of the one-hot dP product at the config-5 shape (V = 256, N = 3H = 6144,
K = 512 x 128 tokens, G = dGh^T / dGi^T bf16, 805 MB) on the streaming kernel (onehot.hip) at
several K-slice counts and on the one-hot gemm_lds kernel, with a plain read of G (torch sum over
rows) as the memory reference.  Median of N launches, events."""
import os, sys, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from gru_mpi_cuda_amd.ops import load_ext

C = load_ext()
dev = torch.device("cuda", 0)
V, H, K = 256, 2048, 512 * 128
N = 3 * H
G = torch.randn(N, K, device=dev).to(torch.bfloat16)
g = torch.Generator(device="cpu").manual_seed(1)
ids = torch.randint(97, 123, (K,), generator=g, dtype=torch.int32)
ids[::9] = 0
ids = ids.to(dev)
s = torch.cuda.current_stream().cuda_stream
out = torch.empty(16 * V * N, device=dev)


def run(fn, n=int(os.environ.get("N", 10))):
    ts = []
    for _ in range(n + 2):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); fn(); e1.record(); torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1000)
    return round(float(np.median(ts[2:])), 1)


def oh(splits, stream, b2=True):
    d = dict(onehot_ids=ids.data_ptr(), B=G.data_ptr(), ldb=K, C=out.data_ptr(), ldc=N, M=V, N=N, K=K,
             splits=splits, algo=2)
    if b2:
        d.update(B2=G.data_ptr(), b2_row=2 * H)
    C.set_gemm_variants(dict(onehot=stream))
    return lambda: C.gemm_nt(d, s)


res = {"G_MB": round(G.numel() * 2 / 1e6, 1)}
res["torch_sum_us"] = run(lambda: G.sum(dim=1))
# GemmVariants.onehot: 1 = 64 columns x 128-token k-tiles, 2 = 32 x 256, 3 = 128 x 64
for geo in (1, 2, 3):
    for sp in [int(x) for x in os.environ.get("SPLITS", "2,4,8").split(",")]:
        res[f"stream_g{geo}_s{sp}_us"] = run(oh(sp, geo))
res["gemm_lds_s8_us"] = run(oh(8, 0))
# row pitch off the power of two: G rows 128 KiB + 128 B apart instead of exactly 128 KiB
PAD = int(os.environ.get("PAD", 64))
Gp = torch.empty(N, K + PAD, device=dev, dtype=torch.bfloat16)
Gp[:, :K] = G
def ohp(splits, geo):
    d = dict(onehot_ids=ids.data_ptr(), B=Gp.data_ptr(), ldb=K + PAD, C=out.data_ptr(), ldc=N, M=V, N=N, K=K,
             splits=splits, algo=2, B2=Gp.data_ptr(), b2_row=2 * H)
    C.set_gemm_variants(dict(onehot=geo))
    return lambda: C.gemm_nt(d, s)
for geo in (1, 2):
    res[f"padded_g{geo}_s8_us"] = run(ohp(8, geo))
res["padded_gemm_lds_s8_us"] = run(ohp(8, 0))
res["torch_sum_padded_us"] = run(lambda: Gp[:, :K].sum(dim=1))
C.set_gemm_variants(dict(onehot=1))
res["best_stream_TBs"] = round(G.numel() * 2 / min(v for k, v in res.items() if k.startswith("stream_")) / 1e6, 2)
res["torch_sum_TBs"] = round(G.numel() * 2 / res["torch_sum_us"] / 1e6, 2)
print(json.dumps(res))
