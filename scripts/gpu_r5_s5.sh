#!/bin/bash
# session 5: generator v2 (distributed sampling, VALU FC, prefetched name tiles): tests + phase probe;
# streaming probe with the recurrences' relaxed hand-off
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 120 --timeout-method thread -k "generator or names" > gpurun_out/s5_tests.log 2>&1
rc=$?; tail -3 gpurun_out/s5_tests.log; [ $rc -ne 0 ] && exit $rc
out=gpurun_out/s5_gen_probe.jsonl; : > $out
for n in 1 8 16 17 32 64; do
  timeout -k 10 120 python scripts/probe_gen_persist.py $n >> $out 2>>gpurun_out/s5_probe.err || exit 1
done
cat $out
timeout -k 10 120 ./scripts/probe_l2_stream 64 > gpurun_out/s5_l2_stream.jsonl 2> gpurun_out/s5_l2_stream.err || exit 1
cat gpurun_out/s5_l2_stream.jsonl
