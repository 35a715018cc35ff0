#!/bin/bash
# fc_xent with LDS-only barriers (weight loads in flight across the softmax): numerics, probe, benches
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread -k "fc or xent or sample or bench_shape or grads" > gpurun_out/fcbar_tests.log 2>&1
rc=$?; tail -2 gpurun_out/fcbar_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python scripts/probe_fc.py || exit 1
H=1024 timeout -k 10 120 python scripts/probe_fc.py || exit 1
for i in 1 2 3; do
  timeout -k 10 300 python bench.py 2>/dev/null | grep '^{' | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["ms_per_step"], d.get("final_loss"))' || exit 1
done
timeout -k 10 300 python bench.py --preset h1024_l2 --per-gpu-batch 128 --steps 30 --warmup 5 2>/dev/null | grep '^{' | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["ms_per_step"], d.get("final_loss"))' || exit 1
