#!/bin/bash
# h2048 step with and without hipBLASLt on one box: bench (alternating) + a kernel trace of each
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for rep in 1 2; do
  for v in 0 1; do
    line=$(GK_BLASLT=$v timeout -k 10 200 python bench.py --preset h2048 --per-gpu-batch 512 --steps 5 --warmup 2 2>/dev/null | grep '^{') || exit 1
    echo "GK_BLASLT=$v $(echo $line | python3 -c 'import json,sys; print(json.load(sys.stdin)["ms_per_step"])')"
  done
done
for v in 0 1; do
  GK_BLASLT=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_h2048_b$v -o run -- python3 bench.py --preset h2048 --per-gpu-batch 512 --steps 3 --warmup 1 > gpurun_out/prof_h2048_b$v.log 2>&1 || exit 1
  python3 scripts/analyze_trace.py gpurun_out/prof_h2048_b$v/run_kernel_trace.csv > gpurun_out/prof_h2048_b$v/summary.txt
  echo "== GK_BLASLT=$v"; head -14 gpurun_out/prof_h2048_b$v/summary.txt
done
