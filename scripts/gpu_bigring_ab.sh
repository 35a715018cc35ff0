#!/bin/bash
# large-H persistent backward with the exchange ring: its tests, then h2048 / h1024_l2 x1024 A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread -k "big or h2048 or wgrad or exchange_ring" > gpurun_out/bigring_tests.log 2>&1
rc=$?; tail -2 gpurun_out/bigring_tests.log; [ $rc -ne 0 ] && exit $rc
run() { local tag=$1; shift
  timeout -k 10 300 python bench.py "$@" 2>/dev/null | grep '^{' | python3 -c "import json,sys; d=json.load(sys.stdin); print(json.dumps({'tag':'$tag','ms':d['ms_per_step'],'loss':d.get('final_loss')}))" | tee -a gpurun_out/bigring_ab.jsonl; }
for i in 1 2; do
  run h2048_r4 --preset h2048 --per-gpu-batch 512 --steps 6 --warmup 2 || exit 1
  run h2048_r0 --preset h2048 --per-gpu-batch 512 --steps 6 --warmup 2 --variant bwd_xring=0 || exit 1
  run h1024x1024_r4 --preset h1024_l2 --per-gpu-batch 1024 --steps 10 --warmup 3 || exit 1
  run h1024x1024_r0 --preset h1024_l2 --per-gpu-batch 1024 --steps 10 --warmup 3 --variant bwd_xring=0 || exit 1
done
