#!/bin/bash
# large-H persistent forward: kernel + engine tests, then h2048 / h1024_l2x1024 benches vs the per-step build
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "fwd_seq_big" > gpurun_out/r4_big_tests.log 2>&1
rc=$?; tail -15 gpurun_out/r4_big_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread -k "big_persistent or lds_step_kernels" > gpurun_out/r4_big_tests2.log 2>&1
rc=$?; tail -5 gpurun_out/r4_big_tests2.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  timeout -k 10 300 python bench.py --preset h2048 --per-gpu-batch 512 --steps 6 --warmup 2 2>/dev/null | grep '^{' | python3 -c 'import json,sys; d=json.load(sys.stdin); print("big", d["ms_per_step"], d["config"]["plan"])' || exit 1
  GK_PERSIST=0 timeout -k 10 300 python bench.py --preset h2048 --per-gpu-batch 512 --steps 6 --warmup 2 2>/dev/null | grep '^{' | python3 -c 'import json,sys; d=json.load(sys.stdin); print("perstep", d["ms_per_step"], d["config"]["plan"])' || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r4_h2048big -o run -- python3 bench.py --preset h2048 --per-gpu-batch 512 --steps 3 --warmup 1 --min-warmup 0 > gpurun_out/prof_r4_h2048big.log 2>&1 || exit 1
python3 scripts/analyze_trace.py gpurun_out/prof_r4_h2048big/run_kernel_trace.csv > gpurun_out/prof_r4_h2048big/summary.txt
head -12 gpurun_out/prof_r4_h2048big/summary.txt
