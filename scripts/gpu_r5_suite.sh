#!/bin/bash
# mid-round check of the whole tree: full GPU suite + smoke + headline driver form
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5_suite.log 2>&1
rc=$?; tail -3 gpurun_out/r5_suite.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5_smoke.log 2>&1
rc=$?; tail -3 gpurun_out/r5_smoke.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 2>/dev/null | grep '^{' >> gpurun_out/r5_suite_bench.jsonl || exit 1
done
cat gpurun_out/r5_suite_bench.jsonl
