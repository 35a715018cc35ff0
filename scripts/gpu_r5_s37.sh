#!/bin/bash
# session 37: counters of the final config-5 and config-4 shards
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
bash scripts/gpu_pmc.sh r5_c5_final --preset h2048 --per-gpu-batch 512 --min-warmup 0 || exit 1
bash scripts/gpu_pmc.sh r5_c4_final --preset h1024_l2 --per-gpu-batch 128 --min-warmup 0 || exit 1
