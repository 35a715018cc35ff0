#!/bin/bash
# h2048 per-step kernel variants, same box, alternating: usage gpu_step_ab.sh TAG "ENV_A" "ENV_B" ... (reps via REPS)
# Each env string is a space-separated list of VAR=value (or "base").
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=$1; shift
out=gpurun_out/ab_$tag.jsonl; : > $out
for i in $(seq ${REPS:-2}); do
  for e in "$@"; do
    line=$(env $( [ "$e" = base ] || echo $e ) timeout -k 10 200 python bench.py --preset h2048 --per-gpu-batch 512 --steps 6 --warmup 2 2>/dev/null | grep '^{') || { echo "run failed ($e)"; exit 1; }
    echo "{\"env\": \"$e\", \"rep\": $i, \"bench\": $line}" >> $out
    echo "$e -> $(echo $line | python3 -c 'import json,sys; print(json.load(sys.stdin)["ms_per_step"])')"
  done
done
