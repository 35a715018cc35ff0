#!/bin/bash
# session 50: generator with in-kernel parity refill of the tagged slots -- tests, probe, timeline of one call
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py tests/test_capi_gpu.py -x -q --timeout 120 --timeout-method thread -k "generator or names or capi or generate" > gpurun_out/s50_tests.log 2>&1
rc=$?; tail -1 gpurun_out/s50_tests.log; [ $rc -ne 0 ] && exit $rc
out=gpurun_out/s50_gen_probe.jsonl; : > $out
for n in 1 8 32; do
  timeout -k 10 120 python scripts/probe_gen_persist.py $n >> $out 2>>gpurun_out/s50_probe.err || exit 1
done
python3 -c "
import json
for l in open('$out'):
    d=json.loads(l); print(d['N'], d['us_per_char'], d['end_to_end_us_per_generate'], d['end_to_end_us_per_char'], d['launch_us']['entry -> loop end'])"
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/prof_gen2 -o run -- python3 scripts/probe_gen_persist.py 1 > gpurun_out/prof_gen2.log 2>&1 || exit 1
ls gpurun_out/prof_gen2
