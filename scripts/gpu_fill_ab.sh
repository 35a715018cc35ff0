#!/bin/bash
# GEMM dispatch wave-fill switch (GK_GEMM256_FILL=0: always the 256x256 kernel for >= 256 tiles) on
# h1024_l2 (128 seq / GPU) and h2048 (512 seq / GPU), alternating on one box
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
b() { local tag=$1 env=$2; shift 2
  line=$(env $env timeout -k 10 300 python bench.py "$@" 2>/dev/null | grep '^{') || { echo "failed $tag"; exit 1; }
  echo "$tag $env $(echo $line | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["ms_per_step"])')"; }
for rep in 1 2 3; do
  b l2 GK_GEMM256_FILL=0.85 --preset h1024_l2 --per-gpu-batch 128 --steps 30 --warmup 5
  b l2 GK_GEMM256_FILL=0 --preset h1024_l2 --per-gpu-batch 128 --steps 30 --warmup 5
done
b h2048 GK_GEMM256_FILL=0.85 --preset h2048 --per-gpu-batch 512 --steps 6 --warmup 2
b h2048 GK_GEMM256_FILL=0 --preset h2048 --per-gpu-batch 512 --steps 6 --warmup 2
exit 0
