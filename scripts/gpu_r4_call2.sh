#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
bash scripts/gpu_r4_big.sh; echo "big rc=$?"
bash scripts/gpu_r4_ab1.sh
