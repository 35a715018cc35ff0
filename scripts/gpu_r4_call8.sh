#!/bin/bash
# single __shared__ object in the large-H persistent kernels (no vmcnt(0) before every ds_read):
# tests, then h2048 / h1024_l2 x 1024 with the persistent forward and backward on / off
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_kernels_gpu.py -x -v --timeout 200 --timeout-method thread -k "big_persistent or wgrad_library or fwd_seq_big" > gpurun_out/r4_c8_tests.log 2>&1
rc=$?; tail -8 gpurun_out/r4_c8_tests.log; [ $rc -ne 0 ] && exit $rc
out=gpurun_out/r4_c8_ab.jsonl
b() { timeout -k 10 300 python bench.py --steps 6 --warmup 2 "$@" 2>/dev/null | grep '^{'; }
for i in 1 2; do
  for v in "fwd_big=0" "fwd_big=1" "bwd_big=0"; do
    l=$(b --preset h2048 --per-gpu-batch 512 --variant $v) || exit 1; echo "{\"form\": \"h2048 $v\", \"bench\": $l}" >> $out
    l=$(b --preset h1024_l2 --per-gpu-batch 1024 --variant $v) || exit 1; echo "{\"form\": \"h1024_l2x1024 $v\", \"bench\": $l}" >> $out
  done
done
python3 -c '
import json
for l in open("'$out'"):
    d = json.loads(l); print(d["form"], d["bench"]["ms_per_step"], d["bench"]["config"].get("plan"))'
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r4_h2048c8 -o run -- python3 bench.py --preset h2048 --per-gpu-batch 512 --steps 3 --warmup 1 --min-warmup 0 --variant fwd_big=1 > gpurun_out/prof_r4_h2048c8.log 2>&1 || exit 1
python3 scripts/analyze_trace.py gpurun_out/prof_r4_h2048c8/run_kernel_trace.csv > gpurun_out/prof_r4_h2048c8/summary.txt
head -12 gpurun_out/prof_r4_h2048c8/summary.txt
