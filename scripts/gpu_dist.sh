#!/bin/bash
# distribution of the driver-form headline bench on one box (final tree)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
out=gpurun_out/final_dist.jsonl; : > $out
for i in 1 2 3 4 5 6; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 2>/dev/null | grep '^{' >> $out || exit 1
  tail -1 $out | python3 -c 'import json,sys; d=json.load(sys.stdin); print("K=20", d["ms_per_step"], d["value"])'
done
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 300 --warmup 50 2>/dev/null | grep '^{' >> $out || exit 1
  tail -1 $out | python3 -c 'import json,sys; d=json.load(sys.stdin); print("K=300", d["ms_per_step"], d["value"])'
done
