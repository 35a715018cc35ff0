#!/bin/bash
# large-H persistent forward + backward: kernel + engine tests, then h2048 benches: both persistent
# (exchange behind an agent acquire), both with sc1 exchange loads, backward only, all per-step
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "fwd_seq_big" > gpurun_out/r4_big_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r4_big_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 200 --timeout-method thread -k "big_persistent" > gpurun_out/r4_big_tests2.log 2>&1
rc=$?; tail -6 gpurun_out/r4_big_tests2.log; [ $rc -ne 0 ] && exit $rc
out=gpurun_out/r4_h2048_big_ab2.jsonl
b() { timeout -k 10 300 python bench.py --preset h2048 --per-gpu-batch 512 --steps 6 --warmup 2 "$@" 2>/dev/null | grep '^{'; }
for i in 1 2; do
  l=$(b) || exit 1; echo "{\"form\": \"big-fwd+bwd acq\", \"bench\": $l}" >> $out
  l=$(b --variant big_acq=0) || exit 1; echo "{\"form\": \"big-fwd+bwd sc1\", \"bench\": $l}" >> $out
  l=$(b --variant fwd_big=0) || exit 1; echo "{\"form\": \"big-bwd acq\", \"bench\": $l}" >> $out
  l=$(GK_PERSIST=0 b) || exit 1; echo "{\"form\": \"per-step\", \"bench\": $l}" >> $out
done
python3 -c '
import json
for l in open("'$out'"):
    d = json.loads(l); print(d["form"], d["bench"]["ms_per_step"], d["bench"]["config"].get("plan"))'
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r4_h2048acq -o run -- python3 bench.py --preset h2048 --per-gpu-batch 512 --steps 3 --warmup 1 --min-warmup 0 > gpurun_out/prof_r4_h2048acq.log 2>&1 || exit 1
python3 scripts/analyze_trace.py gpurun_out/prof_r4_h2048acq/run_kernel_trace.csv > gpurun_out/prof_r4_h2048acq/summary.txt
head -8 gpurun_out/prof_r4_h2048acq/summary.txt
