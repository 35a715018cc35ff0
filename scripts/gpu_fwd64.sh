#!/bin/bash
# persistent 64-row large-H forward: kernel + engine tests, then h2048 / h1024_l2 x 1024 with it on / off
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -v --timeout 200 --timeout-method thread -k "fwd_seq64 or big_persistent" > gpurun_out/fwd64_tests.log 2>&1
rc=$?; tail -9 gpurun_out/fwd64_tests.log; [ $rc -ne 0 ] && exit $rc
out=gpurun_out/fwd64_ab.jsonl
b() { timeout -k 10 300 python bench.py --steps 6 --warmup 2 "$@" 2>/dev/null | grep '^{'; }
for i in 1 2; do
  for v in 1 0; do
    l=$(b --preset h2048 --per-gpu-batch 512 --variant fwd64p=$v) || exit 1; echo "{\"form\": \"h2048 fwd64p=$v\", \"bench\": $l}" >> $out
    l=$(b --preset h1024_l2 --per-gpu-batch 1024 --variant fwd64p=$v) || exit 1; echo "{\"form\": \"h1024_l2x1024 fwd64p=$v\", \"bench\": $l}" >> $out
  done
done
python3 -c '
import json
for l in open("'$out'"):
    d = json.loads(l); print(d["form"], d["bench"]["ms_per_step"], d["bench"]["config"].get("plan"))'
bash scripts/gpu_prof.sh h2048_fwd64 --preset h2048 --per-gpu-batch 512 --steps 3 --warmup 1 --min-warmup 0 | head -8
