#!/bin/bash
# usage: gpu_prof.sh TAG [bench args...]   -> gpurun_out/prof_TAG/
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=$1; shift
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o run -- python3 bench.py --steps 10 --warmup 3 "$@" > gpurun_out/prof_$tag.log 2>&1
rc=$?; echo "prof $tag rc=$rc"; [ $rc -gt 1 ] && exit $rc
python3 scripts/analyze_trace.py gpurun_out/prof_$tag/run_kernel_trace.csv | tee gpurun_out/prof_$tag/summary.txt
