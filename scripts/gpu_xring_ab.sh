#!/bin/bash
# backward exchange ring (bwd_xring=4) vs one slot per step (0): engine tests, then alternating benches
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "bwd or grads or bench_shape or seq" > gpurun_out/xring_tests.log 2>&1
rc=$?; tail -2 gpurun_out/xring_tests.log; [ $rc -ne 0 ] && exit $rc
run() { local tag=$1; shift
  timeout -k 10 300 python bench.py "$@" 2>/dev/null | grep '^{' | python3 -c "import json,sys; d=json.load(sys.stdin); print(json.dumps({'tag':'$tag','ms':d['ms_per_step']}))" | tee -a gpurun_out/xring_ab.jsonl; }
for i in 1 2 3; do
  run h512_ring4 || exit 1
  run h512_ring0 --variant bwd_xring=0 || exit 1
  run c4_ring4 --preset h1024_l2 --per-gpu-batch 128 --steps 30 --warmup 5 || exit 1
  run c4_ring0 --preset h1024_l2 --per-gpu-batch 128 --steps 30 --warmup 5 --variant bwd_xring=0 || exit 1
done
