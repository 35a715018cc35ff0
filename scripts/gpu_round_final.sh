#!/bin/bash
# Round-end evidence, part 1: the full GPU suite and smoke() on the final tree (part 2: gpu_benches.sh)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/final_suite.log 2>&1
rc=$?; tail -2 gpurun_out/final_suite.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final_smoke.log 2>&1
rc=$?; tail -1 gpurun_out/final_smoke.log; exit $rc
