#!/bin/bash
# counters of the final headline step and config-4 shard
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
bash scripts/gpu_pmc.sh r4_h512_final --min-warmup 0 || exit 1
bash scripts/gpu_pmc.sh r4_c4_final --preset h1024_l2 --per-gpu-batch 128 --min-warmup 0 || exit 1
