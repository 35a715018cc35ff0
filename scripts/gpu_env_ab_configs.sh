#!/bin/bash
# Same-box A/B of an environment switch over the headline and the secondary configs, alternating:
# usage gpu_env_ab_configs.sh TAG "ENV_A" "ENV_B" [reps]
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=$1; a=$2; b=$3; reps=${4:-2}
out=gpurun_out/ab_$tag.jsonl; : > $out
configs=("h512|--steps 200 --warmup 20" "h1024_l2_shard|--preset h1024_l2 --per-gpu-batch 128 --steps 50 --warmup 10"
         "h1024_l2_b1024|--preset h1024_l2 --per-gpu-batch 1024 --steps 10 --warmup 3"
         "h2048_b512|--preset h2048 --per-gpu-batch 512 --steps 6 --warmup 2")
for c in "${configs[@]}"; do
  name=${c%%|*}; args=${c#*|}
  for i in $(seq $reps); do
    for e in "$a" "$b"; do
      line=$(env $e timeout -k 10 200 python bench.py $args 2>/dev/null | grep '^{') || { echo "run failed ($name $e)"; exit 1; }
      echo "{\"config\": \"$name\", \"env\": \"$e\", \"rep\": $i, \"bench\": $line}" >> $out
      echo "$name $e -> $(echo $line | python3 -c 'import json,sys; print(json.load(sys.stdin)["ms_per_step"])')"
    done
  done
done
