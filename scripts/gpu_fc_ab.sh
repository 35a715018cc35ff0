#!/bin/bash
# fc_xent: weight-stream issue order rotated per workgroup -- numerics + probe + headline bench
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread -k "fc or xent or sample or bench_shape" > gpurun_out/fc_tests.log 2>&1
rc=$?; tail -2 gpurun_out/fc_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python scripts/probe_fc.py || exit 1
H=1024 M=8192 timeout -k 10 120 python scripts/probe_fc.py || exit 1
for i in 1 2 3; do
  timeout -k 10 300 python bench.py 2>/dev/null | grep '^{' | python3 -c 'import json,sys; print(json.load(sys.stdin)["ms_per_step"])' || exit 1
done
