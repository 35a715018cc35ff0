#!/bin/bash
# Same-box A/B of the weight-gradient GEMM engine (GK_WGRAD_GEMM=256 | lib | 128) on the large
# configs; each line tagged with its engine.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
out=gpurun_out/wgrad_ab.jsonl; : > $out
for rep in 1 2; do
  for eng in 256 lib 128; do
    for cfg in "h2048 --per-gpu-batch 512 --steps 5 --warmup 2" "h1024_l2 --per-gpu-batch 128 --steps 10 --warmup 3"; do
      line=$(GK_WGRAD_GEMM=$eng timeout -k 10 200 python bench.py --preset $cfg 2>/dev/null | grep '^{') || { echo "failed: $eng $cfg"; exit 1; }
      echo "{\"engine\": \"$eng\", \"rep\": $rep, \"bench\": $line}" >> $out
      echo "$eng ${cfg%% *} $(echo $line | python3 -c 'import json,sys; print(json.load(sys.stdin)["ms_per_step"])')"
    done
  done
done
