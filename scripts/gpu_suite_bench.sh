#!/bin/bash
# full GPU suite + smoke + headline / config-4 benches (driver form)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/suite.log 2>&1
rc=$?; tail -2 gpurun_out/suite.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" 2>&1 | tail -1 || exit 1
for i in 1 2 3; do
  timeout -k 10 300 python bench.py 2>/dev/null | grep '^{' | tee -a gpurun_out/suite_bench.jsonl || exit 1
done
timeout -k 10 300 python bench.py --preset h1024_l2 --per-gpu-batch 128 --steps 30 --warmup 5 2>/dev/null | grep '^{' | tee -a gpurun_out/suite_bench.jsonl || exit 1
