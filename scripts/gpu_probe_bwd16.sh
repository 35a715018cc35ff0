#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread -k "bwd16 or grads_match_cpu" > gpurun_out/bwd16_tests.log 2>&1
rc=$?; tail -2 gpurun_out/bwd16_tests.log; [ $rc -ne 0 ] && exit $rc
for cfg in "H=1024 B=128 FW=0 FP=1 R16=1 T=64" "H=1024 B=128 FW=0 FP=0 R16=1 T=64"; do
  env $cfg timeout -k 10 120 python scripts/probe_seq_bwd.py 2>/dev/null | tee -a gpurun_out/probe_bwd16d.jsonl || exit 1
done
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --preset h1024_l2 --per-gpu-batch 128 --steps 30 --warmup 5 2>/dev/null | grep '^{' | python3 -c 'import json,sys; print(json.load(sys.stdin)["ms_per_step"])' || exit 1
done
