#!/bin/bash
# Round-end evidence on the final tree: full GPU suite, smoke, every config's bench, traces
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/final_suite.log 2>&1
rc=$?; tail -2 gpurun_out/final_suite.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" 2>&1 | tail -1 || exit 1
bash scripts/gpu_benches.sh
