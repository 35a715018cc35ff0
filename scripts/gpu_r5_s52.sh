#!/bin/bash
# session 52: h2048 forward step tile, 64-row (default) vs 128-row (--variant fwd64=0), alternating pairs
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
out=gpurun_out/s52_benches.jsonl; : > $out
run() { tag=$1; shift; line=$(timeout -k 10 300 "$@" 2>/dev/null | grep '^{') || { echo "fail $tag"; exit 1; }; echo "{\"tag\": \"$tag\", \"b\": $line}" >> $out; echo "$tag $(echo $line | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["ms_per_step"], d.get("final_loss"))')"; }
for i in 1 2; do
  run c5_fwd64 python bench.py --preset h2048 --per-gpu-batch 512 --steps 6 --warmup 2
  run c5_fwd128 python bench.py --preset h2048 --per-gpu-batch 512 --steps 6 --warmup 2 --variant fwd64=0
done
