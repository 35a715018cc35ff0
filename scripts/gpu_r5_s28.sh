#!/bin/bash
# session 28: tagged layer states on their own lines (N <= 8, H = 1024)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 120 --timeout-method thread -k "generator or names" > gpurun_out/s28_tests.log 2>&1
rc=$?; tail -3 gpurun_out/s28_tests.log; [ $rc -ne 0 ] && exit $rc
out=gpurun_out/s28_gen_probe.jsonl; : > $out
for n in 1 2 8 9 16 64; do
  timeout -k 10 120 python scripts/probe_gen_persist.py $n >> $out 2>>gpurun_out/s28_probe.err || exit 1
done
cat $out
