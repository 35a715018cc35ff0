#!/bin/bash
# session 7: generator v4 (pipelined flag polls, direct logits loads up to 8 names, rolling prefetch at H=1024)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 120 --timeout-method thread -k "generator or names" > gpurun_out/s7_tests.log 2>&1
rc=$?; tail -3 gpurun_out/s7_tests.log; [ $rc -ne 0 ] && exit $rc
out=gpurun_out/s7_gen_probe.jsonl; : > $out
for n in 1 8 16 17 32 64; do
  timeout -k 10 120 python scripts/probe_gen_persist.py $n >> $out 2>>gpurun_out/s7_probe.err || exit 1
done
cat $out
