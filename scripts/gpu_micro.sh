#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 200 python scripts/microbench_launch.py > gpurun_out/micro.log 2>&1; echo "micro rc=$?"; tail -2 gpurun_out/micro.log
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-graph > gpurun_out/bench_nograph.log 2>&1; echo "nograph rc=$?"; tail -1 gpurun_out/bench_nograph.log
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --chunks 1 > gpurun_out/bench_c1.log 2>&1; echo "c1 rc=$?"; tail -1 gpurun_out/bench_c1.log
