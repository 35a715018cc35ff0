#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 200 python bench.py > gpurun_out/r4_base_default.json 2>gpurun_out/r4_base_default.err || { tail -20 gpurun_out/r4_base_default.err; exit 1; }
cat gpurun_out/r4_base_default.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r4_h512 -o run -- python3 bench.py --steps 10 --warmup 3 --min-warmup 50 > gpurun_out/prof_r4_h512.log 2>&1 || exit 1
python3 scripts/analyze_trace.py gpurun_out/prof_r4_h512/run_kernel_trace.csv > gpurun_out/prof_r4_h512/summary.txt
cat gpurun_out/prof_r4_h512/summary.txt
bash scripts/gpu_r4_gemm.sh || exit 1
timeout -k 10 300 python bench.py --preset h2048 --per-gpu-batch 512 --steps 6 --warmup 2 > gpurun_out/r4_base_h2048.json 2>&1 || exit 1
tail -1 gpurun_out/r4_base_h2048.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r4_h2048 -o run -- python3 bench.py --preset h2048 --per-gpu-batch 512 --steps 3 --warmup 1 --min-warmup 0 > gpurun_out/prof_r4_h2048.log 2>&1 || exit 1
python3 scripts/analyze_trace.py gpurun_out/prof_r4_h2048/run_kernel_trace.csv > gpurun_out/prof_r4_h2048/summary.txt
head -20 gpurun_out/prof_r4_h2048/summary.txt
bash scripts/gpu_r4_h2048_ab.sh
