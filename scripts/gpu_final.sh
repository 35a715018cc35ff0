#!/bin/bash
# Round-end evidence: GPU suite, smoke, the benches of every config, a headline trace.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
bash scripts/gpu_full_suite.sh || exit 1
bash scripts/gpu_benches.sh
