#!/bin/bash
# usage: gpu_prof_gen.sh TAG [bench_generate args...] -> gpurun_out/profgen_TAG/ (kernel trace summary)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=$1; shift
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profgen_$tag -o run -- python3 bench/bench_generate.py --modes engine "$@" > gpurun_out/profgen_$tag.log 2>&1
rc=$?; echo "profgen $tag rc=$rc"; tail -2 gpurun_out/profgen_$tag.log; [ $rc -gt 1 ] && exit $rc
python3 scripts/analyze_trace.py gpurun_out/profgen_$tag/run_kernel_trace.csv --all | tee gpurun_out/profgen_$tag/summary.txt
