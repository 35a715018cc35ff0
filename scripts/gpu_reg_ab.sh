#!/bin/bash
# same-box A/B: round-2 final tree (_old/, 432dd48) vs the current tree on the large configs
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
out=gpurun_out/reg_ab.jsonl; : > $out
run() {
  local tag=$1 dir=$2; shift 2
  line=$(cd $dir && timeout -k 10 300 python bench.py "$@" 2>/dev/null | grep '^{') || { echo "run failed ($tag)"; exit 1; }
  echo "{\"tag\": \"$tag\", \"bench\": $line}" >> $out
  echo "$tag -> $(echo $line | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["ms_per_step"])')"
}
for i in 1 2; do
  run old_h2048 _old --preset h2048 --per-gpu-batch 512 --steps 6 --warmup 2
  run new_h2048 . --preset h2048 --per-gpu-batch 512 --steps 6 --warmup 2
  run old_b1024 _old --preset h1024_l2 --per-gpu-batch 1024 --steps 10 --warmup 3
  run new_b1024 . --preset h1024_l2 --per-gpu-batch 1024 --steps 10 --warmup 3
  run old_shard _old --preset h1024_l2 --per-gpu-batch 128 --steps 50 --warmup 10
  run new_shard . --preset h1024_l2 --per-gpu-batch 128 --steps 50 --warmup 10
done
