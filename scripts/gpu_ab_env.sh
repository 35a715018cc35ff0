#!/bin/bash
# Same-box A/B of an environment switch on the headline bench: usage gpu_ab_env.sh TAG "ENV_A" "ENV_B" [reps]
# (alternating A B A B ... runs of bench.py --steps 200; each line tagged with its env)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
tag=$1; a=$2; b=$3; reps=${4:-3}
out=gpurun_out/ab_$tag.jsonl; : > $out
for i in $(seq $reps); do
  for e in "$a" "$b"; do
    line=$(env $e timeout -k 10 120 python bench.py --steps 200 --warmup 20 2>/dev/null | grep '^{') || { echo "run failed ($e)"; exit 1; }
    echo "{\"env\": \"$e\", \"rep\": $i, \"bench\": $line}" >> $out
    echo "$e -> $(echo $line | python3 -c 'import json,sys; print(json.load(sys.stdin)["ms_per_step"])')"
  done
done
