#!/bin/bash
# spin-budget fix (clock-only first check) + large-H acquire exchange: tests, h2048 A/B, headline vs r3
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
bash scripts/gpu_r4_big.sh || exit 1
bash scripts/gpu_multi_ab.sh "new ab_r3" 3 gpurun_out/r4_ab3_driver.jsonl --steps 20 --warmup 5 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r4_h512d -o run -- python3 bench.py --steps 10 --warmup 3 --min-warmup 50 > gpurun_out/prof_r4_h512d.log 2>&1 || exit 1
python3 scripts/analyze_trace.py gpurun_out/prof_r4_h512d/run_kernel_trace.csv > gpurun_out/prof_r4_h512d/summary.txt
cat gpurun_out/prof_r4_h512d/summary.txt
