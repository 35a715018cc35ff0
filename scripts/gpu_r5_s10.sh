#!/bin/bash
# session 10: 4-wave 128 x 128-per-wave gemm256 (GK_GEMM256_W4=1): tests, then GEMM bench against
# the phased / legacy 8-wave kernels and hipBLASLt
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "gemm256" > gpurun_out/s10_tests.log 2>&1
rc=$?; tail -3 gpurun_out/s10_tests.log; [ $rc -ne 0 ] && exit $rc
GEMM_ONLY256=1 GEMM_SHAPES=h2048.dW_hh,sq8192,sq4096,h1024.dWih,h1024.Gi timeout -k 10 400 python -u scripts/bench_gemm.py > gpurun_out/s10_gemm.jsonl 2> gpurun_out/s10_gemm.err || exit 1
python3 -c "
import json
for l in open('gpurun_out/s10_gemm.jsonl'):
    d=json.loads(l); print(d['shape'], {k:v for k,v in d.items() if k.endswith('tflops')})"
