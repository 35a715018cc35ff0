#!/bin/bash
# h2048 shard: split-K backward block order A/B (bwd_sk_map 0 vs 1), alternating, + kernel test
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
out=gpurun_out/r4_h2048_skmap.jsonl; : > $out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "bwd_step_sk" > gpurun_out/r4_skmap_tests.log 2>&1 || { tail -5 gpurun_out/r4_skmap_tests.log; exit 1; }
tail -1 gpurun_out/r4_skmap_tests.log
for rep in 1 2; do
for m in 0 1; do
  line=$(timeout -k 10 300 python bench.py --preset h2048 --per-gpu-batch 512 --steps 6 --warmup 2 --variant bwd_sk_map=$m 2>/dev/null | grep '^{') || exit 1
  echo "{\"bwd_sk_map\": $m, \"bench\": $line}" >> $out
  echo "map=$m $(echo $line | python3 -c 'import json,sys; print(json.load(sys.stdin)["ms_per_step"])')"
done
done
