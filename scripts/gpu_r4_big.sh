#!/bin/bash
# large-H persistent forward + backward: kernel + engine tests, then h2048 benches: both persistent,
# forward only (bwd_big=0), all per-step (GK_PERSIST=0); then a kernel trace of the default
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "fwd_seq_big" > gpurun_out/r4_big_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r4_big_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 200 --timeout-method thread -k "big_persistent" > gpurun_out/r4_big_tests2.log 2>&1
rc=$?; tail -6 gpurun_out/r4_big_tests2.log; [ $rc -ne 0 ] && exit $rc
b() { timeout -k 10 300 python bench.py --preset h2048 --per-gpu-batch 512 --steps 6 --warmup 2 "$@" 2>/dev/null | grep '^{'; }
for i in 1 2; do
  l=$(b) || exit 1; echo "{\"form\": \"big-fwd+bwd\", \"bench\": $l}" >> gpurun_out/r4_h2048_big_ab.jsonl
  l=$(b --variant bwd_big=0) || exit 1; echo "{\"form\": \"big-fwd\", \"bench\": $l}" >> gpurun_out/r4_h2048_big_ab.jsonl
  l=$(GK_PERSIST=0 b) || exit 1; echo "{\"form\": \"per-step\", \"bench\": $l}" >> gpurun_out/r4_h2048_big_ab.jsonl
done
python3 -c '
import json
for l in open("gpurun_out/r4_h2048_big_ab.jsonl"):
    d = json.loads(l); print(d["form"], d["bench"]["ms_per_step"], d["bench"]["config"].get("plan"))'
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r4_h2048big -o run -- python3 bench.py --preset h2048 --per-gpu-batch 512 --steps 3 --warmup 1 --min-warmup 0 > gpurun_out/prof_r4_h2048big.log 2>&1 || exit 1
python3 scripts/analyze_trace.py gpurun_out/prof_r4_h2048big/run_kernel_trace.csv > gpurun_out/prof_r4_h2048big/summary.txt
head -14 gpurun_out/prof_r4_h2048big/summary.txt
