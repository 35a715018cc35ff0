#!/bin/bash
# session 26: dW_fc on gemm256p -- kernel check at the config-5 shape, engine gradient comparison
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 200 python -u - <<'PY' > gpurun_out/s26_kernel.log 2>&1
import torch
from gru_mpi_cuda_amd.ops import load_ext
C = load_ext(); s = torch.cuda.current_stream().cuda_stream
for (M, N, K, sp, ldb_pad) in [(256, 2048, 65536, 32, 512), (256, 2048, 65536, 8, 0), (256, 256, 65536, 32, 512)]:
    A = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
    Bf = (torch.rand(N, K + ldb_pad, device="cuda") * 2 - 1).bfloat16()
    B = Bf[:, ldb_pad:]
    out = torch.full((sp, M, N), float("nan"), device="cuda"); rs = torch.full((sp, M), float("nan"), device="cuda")
    for algo in (5, 2):
        d = dict(A=A.data_ptr(), lda=K, B=B.data_ptr(), ldb=K + ldb_pad, C=out.data_ptr(), ldc=N, M=M, N=N, K=K, splits=sp, algo=algo, rowsumA=rs.data_ptr())
        try:
            C.gemm_nt(d, s)
        except RuntimeError as e:
            print(M, N, K, sp, algo, "refused", str(e)[:80]); continue
        torch.cuda.synchronize()
        ref = A.float() @ B.float().T
        e1 = float((out.sum(0) - ref).abs().max() / ref.abs().max()); e2 = float((rs.sum(0) - A.float().sum(1)).abs().max() / A.float().sum(1).abs().max())
        print(M, N, K, sp, ldb_pad, "algo", algo, "C relerr", f"{e1:.2e}", "rowsum relerr", f"{e2:.2e}", flush=True)
PY
rc=$?; cat gpurun_out/s26_kernel.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 120 --timeout-method thread -k "dwfc_gemm256" > gpurun_out/s26_tests.log 2>&1
rc=$?; tail -5 gpurun_out/s26_tests.log; exit $rc
