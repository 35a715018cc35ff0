#!/bin/bash
# backward per-step phases at H=1024 (no fused dW_hh), local vs write-through hand-off, 4 vs 8 row blocks
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
out=gpurun_out/bwd_loc.jsonl; : > $out
for cfg in "1024 128 1" "1024 256 1" "1024 256 0" "512 256 1" "512 256 0"; do
  set -- $cfg
  fw=1; [ $1 -ge 1024 ] && fw=0
  H=$1 B=$2 LOCAL=$3 FW=$fw FP=1 timeout -k 10 120 python scripts/probe_seq_bwd.py >> $out 2>/dev/null || { echo "probe failed $cfg"; exit 1; }
  tail -1 $out
done
