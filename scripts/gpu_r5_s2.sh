#!/bin/bash
# session 2: phased GEMM v2 (tests + bench), the pipelined DP tail's timeline at one rank
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "gemm256 or wgrad or exchange_ring" > gpurun_out/s2_tests.log 2>&1
rc=$?; tail -2 gpurun_out/s2_tests.log; [ $rc -ne 0 ] && exit $rc
GEMM_ONLY256=1 GEMM_SHAPES=h2048.dW_hh,sq8192,sq4096,h1024.dWih,h1024.Gi,h2048.dH timeout -k 10 300 python -u scripts/bench_gemm.py > gpurun_out/gemm_bench_v2.jsonl 2> gpurun_out/gemm_bench.err || exit 1
python3 -c "
import json
for l in open('gpurun_out/gemm_bench_v2.jsonl'):
    d=json.loads(l); print(d['shape'], {k:v for k,v in d.items() if k.endswith('tflops')})"
for m in 1 0; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_dp$m -o run -- python3 bench.py --steps 10 --warmup 3 --rccl-self --dp-pipeline $m > gpurun_out/prof_dp$m.log 2>&1 || exit 1
  python3 scripts/analyze_trace.py gpurun_out/prof_dp$m/run_kernel_trace.csv --prologue --timeline > gpurun_out/prof_dp$m/summary.txt
  head -40 gpurun_out/prof_dp$m/summary.txt
done
