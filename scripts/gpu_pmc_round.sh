#!/bin/bash
# hardware counters of the h2048 shard and the h512 headline step (profiles/rN_*_pmc_summary.txt)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
bash scripts/gpu_pmc.sh r4_h2048 --preset h2048 --per-gpu-batch 512 --min-warmup 0 || exit 1
bash scripts/gpu_pmc.sh r4_h512 --min-warmup 0 || exit 1
