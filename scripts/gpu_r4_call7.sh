#!/bin/bash
# fused bias partials in the large-H backward + auto library dW_hh: tests, h2048 / h1024_l2 benches, trace
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 200 --timeout-method thread -k "big_persistent or dwfc or bench_shape or wgrad_library" > gpurun_out/r4_c7_tests.log 2>&1
rc=$?; tail -7 gpurun_out/r4_c7_tests.log; [ $rc -ne 0 ] && exit $rc
out=gpurun_out/r4_c7_ab.jsonl
b() { timeout -k 10 300 python bench.py --steps 6 --warmup 2 "$@" 2>/dev/null | grep '^{'; }
for i in 1 2; do
  l=$(b --preset h2048 --per-gpu-batch 512) || exit 1; echo "{\"form\": \"h2048 default\", \"bench\": $l}" >> $out
  l=$(GK_WGRAD_GEMM=256 b --preset h2048 --per-gpu-batch 512) || exit 1; echo "{\"form\": \"h2048 GK_WGRAD_GEMM=256\", \"bench\": $l}" >> $out
  l=$(b --preset h1024_l2 --per-gpu-batch 1024) || exit 1; echo "{\"form\": \"h1024_l2 x1024 default\", \"bench\": $l}" >> $out
  l=$(b --preset h1024_l2 --per-gpu-batch 1024 --variant bwd_big=0) || exit 1; echo "{\"form\": \"h1024_l2 x1024 bwd_big=0\", \"bench\": $l}" >> $out
done
python3 -c '
import json
for l in open("'$out'"):
    d = json.loads(l); print(d["form"], d["bench"]["ms_per_step"], d["bench"]["config"].get("plan"))'
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r4_h2048c7 -o run -- python3 bench.py --preset h2048 --per-gpu-batch 512 --steps 3 --warmup 1 --min-warmup 0 > gpurun_out/prof_r4_h2048c7.log 2>&1 || exit 1
python3 scripts/analyze_trace.py gpurun_out/prof_r4_h2048c7/run_kernel_trace.csv > gpurun_out/prof_r4_h2048c7/summary.txt
head -16 gpurun_out/prof_r4_h2048c7/summary.txt
