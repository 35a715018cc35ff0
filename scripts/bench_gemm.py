"""GEMM microbenchmark on the engine's shapes: register-direct 64x64 kernel (algo 1), LDS-staged
128x128 (algo 2), hipBLASLt through the engine's wrapper (algo 4), LDS-staged 256x256 (algo 5, at
several split-K depths) and torch (hipBLASLt).  Random uniform [-1,1) bf16 operands (guide rule 25).
GEMM_SHAPES=name1,name2 restricts the run."""
import os, sys, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from gru_mpi_cuda_amd.ops import load_ext

C = load_ext()
dev = torch.device("cuda", 0)
s = torch.cuda.current_stream().cuda_stream
SHAPES = [  # (name, M, N, K, splits)
    ("h512.dH", 8192, 512, 256, 1),
    ("h512.P", 256, 1536, 512, 1),
    ("h512.dEmb", 256, 512, 1536, 1),
    ("h512.dW_ih0", 1536, 512, 256, 1),
    ("h512.dW_fc", 256, 512, 8192, 8),
    ("h512.dW_hh", 1536, 512, 8192, 8),
    ("h1024.Gi", 8192, 3072, 1024, 1),
    ("h1024.dWih", 3072, 1024, 8192, 8),
    ("h2048.dW_hh", 6144, 2048, 65536, 8),
    ("h2048.dH", 65536, 2048, 256, 1),
    ("h2048.logits", 65536, 256, 2048, 1),
    ("h2048.dW_fc", 256, 2048, 65536, 32),
    ("h1024.dW_fc", 256, 1024, 8192, 8),
    ("h2048.dW_ih0", 6144, 2048, 256, 1),
    ("h2048.P", 256, 6144, 2048, 1),
    ("h2048.dEmb", 256, 2048, 6144, 8),
    ("h1024.dW_hh", 3072, 1024, 8192, 4),
    ("h1024.dX", 8192, 1024, 3072, 1),
    ("sq4096", 4096, 4096, 4096, 1),
    ("sq8192", 8192, 8192, 8192, 1),
    ("h2048.step_fwd", 512, 6144, 2048, 1),
    ("h2048.step_bwd", 512, 2048, 6144, 1),
    ("h1024.step_bwd_b1024", 1024, 1024, 3072, 1),
]
if os.environ.get("GEMM_SHAPES"):
    keep = set(os.environ["GEMM_SHAPES"].split(","))
    SHAPES = [s for s in SHAPES if s[0] in keep]


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(n):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); fn(); e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    return float(np.median(ts))


res = []
for name, M, N, K, sp in SHAPES:
    A = (torch.rand(M, K, device=dev) * 2 - 1).bfloat16()
    B = (torch.rand(N, K, device=dev) * 2 - 1).bfloat16()
    Cs = torch.empty(sp, M, N, device=dev)
    flop = 2.0 * M * N * K
    row = {"shape": name, "M": M, "N": N, "K": K, "splits": sp}
    ref = (A.float() @ B.float().T) if M * N * K <= 2 ** 41 else None
    variants = [(1, sp), (2, sp), (4, 1)] + [(5, k) for k in (1, 2, 4, 8) if K % (64 * k) == 0 and (k == 1 or K >= 4096)]
    # the 128 x 128 kernel at other split-K depths (GEMM_SPLITS2=8,16,..)
    variants += [(2, int(k)) for k in os.environ.get("GEMM_SPLITS2", "").split(",") if k and int(k) != sp]
    # algo 3: the one-shot small GEMM at the K-slices it takes (h512 step products)
    variants += [(3, k) for k in (1, 2, 4, 6, 8, 16) if K % k == 0 and (K // k) in (128, 192, 256, 512, 1024, 1536, 2048)]
    # algo "5m": the 256 x 256 kernel on v_mfma_f32_32x32x16_bf16 (GemmVariants mfma = 32); "5o": the
    # one-vmcnt(0)-per-k-tile 16x16 kernel (phased = 0) against the phased default
    # "5r": the phased kernel with the fused row sums of A (the weight-gradient form)
    variants += ([("5m", k) for a_, k in variants if a_ == 5] + [("5o", k) for a_, k in variants if a_ == 5]
                 + [("5r", k) for a_, k in variants if a_ == 5]
                 + [(x, k) for a_, k in variants if a_ == 5 for x in ("5g", "5h", "5i", "5")])
    if os.environ.get("GEMM_ONLY256"):
        variants = [v for v in variants if v[0] in (5, "5", "5g", "5h", "5i")]
    for algo, ks in variants:
        C.set_gemm_variants(dict(mfma=32 if algo == "5m" else 16, phased=0 if algo == "5o" else 1,
                                 sched=-1,   # the staggered schedule picked per shape
                                 groupm={"5g": 8, "5h": 16, "5i": 2}.get(algo, 4)))
        algo_arg = 5 if algo in ("5m", "5o", "5r", "5", "5g", "5h", "5i") else algo
        if ks > 1 and Cs.shape[0] < ks:
            Cs = torch.empty(ks, M, N, device=dev)
        d = dict(A=A.data_ptr(), lda=K, B=B.data_ptr(), ldb=K, C=Cs.data_ptr(), ldc=N, M=M, N=N, K=K,
                 splits=ks, algo=algo_arg)
        if algo == "5r":
            rs = torch.empty(ks, M, device=dev)
            d["rowsumA"] = rs.data_ptr()
        tag = f"algo{algo}" + (f"s{ks}" if algo_arg in (3, 5) or (algo_arg == 2 and ks != sp) else "")
        if tag in row or f"{tag}_us" in row:
            tag += "b"   # a repeated variant (order check)
        try:
            us = timeit(lambda: C.gemm_nt(d, s))
        except RuntimeError as e:
            row[tag] = str(e)[:60]
            continue
        row[f"{tag}_us"] = round(us, 1)
        row[f"{tag}_tflops"] = round(flop / us / 1e6, 1)
        if ref is not None:
            err = float((Cs[:ks].sum(0) - ref).abs().max() / ref.abs().max())
            row[f"{tag}_relerr"] = float(f"{err:.2e}")
    us = timeit(lambda: A @ B.T)
    row["torch_us"] = round(us, 1)
    row["torch_tflops"] = round(flop / us / 1e6, 1)
    res.append(row)
    print(json.dumps(row), flush=True)
