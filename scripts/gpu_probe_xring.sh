#!/bin/bash
# 16-row backward: T-deep exchange vs a reused ring of slots (per-phase probe, config-4 shape)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for xr in 0 2 4 0 2 4; do
  for fp in 1 0; do
    XR=$xr H=1024 B=128 FW=0 FP=$fp R16=1 T=64 timeout -k 10 120 python scripts/probe_seq_bwd.py 2>/dev/null | tee -a gpurun_out/probe_xring.jsonl || exit 1
  done
done
