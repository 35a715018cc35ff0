#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
bash scripts/gpu_multi_ab.sh "new ab_r3 ab_dyb" 3 gpurun_out/r4_ab1_driver.jsonl --steps 20 --warmup 5 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r4_h512b -o run -- python3 bench.py --steps 10 --warmup 3 --min-warmup 50 > gpurun_out/prof_r4_h512b.log 2>&1 || exit 1
python3 scripts/analyze_trace.py gpurun_out/prof_r4_h512b/run_kernel_trace.csv > gpurun_out/prof_r4_h512b/summary.txt
cat gpurun_out/prof_r4_h512b/summary.txt
