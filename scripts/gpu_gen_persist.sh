#!/bin/bash
# Persistent small-batch fp32 generation: GPU tests, then chars/s vs the batched fp32 / bf16 paths.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 120 --timeout-method thread \
  -k "persistent or generator" > gpurun_out/gp_tests.log 2>&1
rc=$?; tail -25 gpurun_out/gp_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench/bench_generate.py --modes engine_fp32,engine_fp32_batched,engine --names 1,8,16,32,64 --reps 10 > gpurun_out/gp_bench.log 2>&1
rc=$?; cat gpurun_out/gp_bench.log | tail -20; exit $rc
