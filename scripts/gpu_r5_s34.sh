#!/bin/bash
# session 34: gates + publishes by wave 0 alone up to 16 names -- generator tests, probe
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 120 --timeout-method thread -k "generator or names" > gpurun_out/s34_tests.log 2>&1
rc=$?; tail -2 gpurun_out/s34_tests.log; [ $rc -ne 0 ] && exit $rc
out=gpurun_out/s34_gen_probe.jsonl; : > $out
for n in 1 2 8 9 16 17 32 64; do
  timeout -k 10 120 python scripts/probe_gen_persist.py $n >> $out 2>>gpurun_out/s34_probe.err || exit 1
done
python3 -c "
import json
for l in open('$out'):
    d=json.loads(l); print(d['N'], d['us_per_char'], d['sclk_ghz'], d['phase_us'], d['L1_phase_us'])"
