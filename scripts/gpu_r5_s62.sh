#!/bin/bash
# session 62: final-tree headline kernel trace and counters
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/s62_trace -o run -- python3 bench.py --steps 10 --warmup 2 --graph-steps 1 > gpurun_out/s62_trace.log 2>&1 || exit 1
python3 scripts/analyze_trace.py gpurun_out/s62_trace/run_kernel_trace.csv --prologue > gpurun_out/s62_trace/summary.txt
head -10 gpurun_out/s62_trace/summary.txt
bash scripts/gpu_pmc.sh r5_h512_final --min-warmup 0 || exit 1
