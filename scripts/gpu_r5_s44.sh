#!/bin/bash
# session 44: staggered GEMM priority placement A/B (GK_GEMM256_PRIO 0 MFMA at prio 1, 1 none, 2 R segments at prio 1)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for pr in 1 2; do
  GK_GEMM256_PRIO=$pr timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "gemm256" > gpurun_out/s44_tests_$pr.log 2>&1
  rc=$?; tail -1 gpurun_out/s44_tests_$pr.log; [ $rc -ne 0 ] && exit $rc
done
GEMM_ONLY256=1 GEMM_SHAPES=sq8192,sq4096,h2048.dW_hh timeout -k 10 500 python -u scripts/bench_gemm.py > gpurun_out/s44_gemm.jsonl 2> gpurun_out/s44_gemm.err || exit 1
python3 -c "
import json
for l in open('gpurun_out/s44_gemm.jsonl'):
    d=json.loads(l); print(d['shape'], {k[:-7]:v for k,v in d.items() if k.endswith('tflops') and ('s1_' in k or 's1' == k[-9:-7] or k.startswith('torch'))})"
