#!/bin/bash
# gemm256 on 32x32x16 vs 16x16x32: numerics tests + microbench on the big shapes
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k gemm256 > gpurun_out/g32_tests.log 2>&1; rc=$?; tail -2 gpurun_out/g32_tests.log; [ $rc -ne 0 ] && { grep -E "^E " gpurun_out/g32_tests.log | head; exit $rc; }
GEMM_ONLY256=1 GEMM_SHAPES=sq4096,sq8192,h2048.dW_hh,h1024.Gi,h1024.dWih,h2048.dH timeout -k 10 400 python scripts/bench_gemm.py > gpurun_out/g32_bench.jsonl || exit 1
python3 - <<'PY'
import json
for l in open("gpurun_out/g32_bench.jsonl"):
    r = json.loads(l)
    print(r["shape"], {k: v for k, v in r.items() if k.endswith("_tflops")})
PY
