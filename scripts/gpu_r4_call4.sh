#!/bin/bash
# round-4 hardware counters: h2048 shard (persistent large-H kernels) and the h512 headline step
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
bash scripts/gpu_pmc.sh r4_h2048 --preset h2048 --per-gpu-batch 512 --min-warmup 0 || exit 1
bash scripts/gpu_pmc.sh r4_h512 --min-warmup 0 || exit 1
