#!/bin/bash
# gemm256 forms (16x16x32 2-buffer, 32x32x16, 4-deep 32-k ring) vs hipBLASLt on the engine's large shapes
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "gemm256" > gpurun_out/r4_gemm_tests.log 2>&1 || { tail -20 gpurun_out/r4_gemm_tests.log; exit 1; }
tail -1 gpurun_out/r4_gemm_tests.log
GEMM_ONLY256=1 GEMM_SHAPES=h2048.dW_hh,sq8192,sq4096,h1024.dWih,h1024.Gi timeout -k 10 300 python scripts/bench_gemm.py > gpurun_out/r4_gemm256r.jsonl 2>&1 || exit 1
python3 - <<'PY'
import json
for l in open("gpurun_out/r4_gemm256r.jsonl"):
    if not l.startswith("{"): continue
    d = json.loads(l)
    print(d["shape"], {k: v for k, v in d.items() if k.endswith("tflops")})
PY
