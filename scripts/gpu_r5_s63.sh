#!/bin/bash
# session 63: final-tree headline kernel trace in the driver's form (1 lead step + a 19-step graph)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/s63_trace -o run -- python3 bench.py --steps 20 --warmup 5 > gpurun_out/s63_trace.log 2>&1 || exit 1
tail -1 gpurun_out/s63_trace.log
