#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 200 --timeout-method thread -k "dwfc_gemm256" > gpurun_out/dwfc256_tests.log 2>&1
rc=$?; tail -3 gpurun_out/dwfc256_tests.log; [ $rc -ne 0 ] && exit $rc
out=gpurun_out/dwfc256_ab.jsonl
for i in 1 2; do
  for v in 1 0; do
    l=$(timeout -k 10 300 python bench.py --preset h2048 --per-gpu-batch 512 --steps 6 --warmup 2 --variant dwfc256=$v 2>/dev/null | grep '^{') || exit 1
    echo "{\"dwfc256\": $v, \"bench\": $l}" >> $out
    echo "dwfc256=$v $(echo $l | python3 -c 'import json,sys; print(json.load(sys.stdin)["ms_per_step"])')"
  done
done
bash scripts/gpu_prof.sh h2048_dwfc256 --preset h2048 --per-gpu-batch 512 --steps 3 --warmup 1 --min-warmup 0 | head -12
