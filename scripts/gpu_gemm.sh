#!/bin/bash
# gemm256 phased pipeline: correctness tests, then the GEMM bench on the large shapes
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "gemm256" -x -q --timeout 120 --timeout-method thread > gpurun_out/gemm_test.log 2>&1
rc=$?; tail -3 gpurun_out/gemm_test.log; [ $rc -ne 0 ] && exit $rc
GEMM_ONLY256=1 GEMM_SHAPES=h2048.dW_hh,sq8192,sq4096,h1024.dWih,h1024.Gi,h2048.dH timeout -k 10 300 python -u scripts/bench_gemm.py > gpurun_out/gemm_bench.jsonl 2> gpurun_out/gemm_bench.err
rc=$?; cat gpurun_out/gemm_bench.jsonl; exit $rc
