#!/bin/bash
# kernel-trace profiles of the headline step + timed runs of the other BASELINE configs
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
bash scripts/gpu_prof.sh h512 || exit $?
bash scripts/gpu_prof.sh h1024l2 --preset h1024_l2 --per-gpu-batch 128 || exit $?
for p in "h1024_l2 --per-gpu-batch 128" "h2048 --per-gpu-batch 512"; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --preset $p > gpurun_out/bench_${p%% *}.log 2>&1
  rc=$?; echo "bench $p rc=$rc"; tail -1 gpurun_out/bench_${p%% *}.log; [ $rc -gt 1 ] && exit $rc
done
exit 0
