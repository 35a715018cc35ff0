#!/bin/bash
# session 59: generator error word stored to host-coherent memory by the kernel's last workgroup
# (GK_GEN_ERRCOPY=0) vs a pinned D2H copy after the launch (1) -- tests, end-to-end probe alternating
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py tests/test_capi_gpu.py -x -q --timeout 120 --timeout-method thread -k "generator or names or capi or generate" > gpurun_out/s59_tests.log 2>&1
rc=$?; tail -1 gpurun_out/s59_tests.log; [ $rc -ne 0 ] && exit $rc
out=gpurun_out/s59_gen_probe.jsonl; : > $out
for i in 1 2; do
  for n in 1 8 64; do
    for pin in 1 0; do
      GK_GEN_ERRCOPY=$pin timeout -k 10 120 python scripts/probe_gen_persist.py $n > gpurun_out/s59_one.json 2>>gpurun_out/s59_probe.err || exit 1
      python3 -c "
import json
d=json.load(open('gpurun_out/s59_one.json')); d['errcopy']=$pin; print(json.dumps(d))" >> $out
    done
  done
done
python3 -c "
import json
for l in open('$out'):
    d=json.loads(l); print(d['N'], 'errcopy', d['errcopy'], d['us_per_char'], d['end_to_end_us_per_generate'], d['end_to_end_us_per_char'])"
