#!/bin/bash
# round-end evidence + the backward hand-off protocol probe at H=512 (local vs write-through)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
bash scripts/gpu_round_end.sh || exit 1
out=gpurun_out/bwd_loc.jsonl; : > $out
for L in 1 0; do
  H=512 B=256 LOCAL=$L FW=1 FP=1 timeout -k 10 120 python scripts/probe_seq_bwd.py >> $out 2>/dev/null || exit 1
  tail -1 $out
done
