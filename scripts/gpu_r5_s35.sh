#!/bin/bash
# session 35: staggered GEMM -- A pieces 2.. of k-tile kt+2 in R1(kt+1) (GK_GEMM256_SCHED=1) vs all in R4(kt)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for sc in 0 1; do
  GK_GEMM256_SCHED=$sc timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "gemm256" > gpurun_out/s35_tests_$sc.log 2>&1
  rc=$?; tail -1 gpurun_out/s35_tests_$sc.log; [ $rc -ne 0 ] && exit $rc
done
GEMM_ONLY256=1 GEMM_SHAPES=h2048.dW_hh,h1024.dWih,sq8192,sq4096 timeout -k 10 500 python -u scripts/bench_gemm.py > gpurun_out/s35_gemm.jsonl 2> gpurun_out/s35_gemm.err || exit 1
python3 -c "
import json
for l in open('gpurun_out/s35_gemm.jsonl'):
    d=json.loads(l); print(d['shape'], {k[:-7]:v for k,v in d.items() if k.endswith('tflops') and ('5s' in k or '5b' in k or '5r' in k or 'torch' in k)})
    print('  maxrelerr', max(v for k,v in d.items() if k.endswith('relerr')))"
