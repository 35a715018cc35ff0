#!/bin/bash
# Round-5 start: headline bench x3 + kernel trace of the headline step on the current tree
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
out=gpurun_out/r5_base.jsonl; : > $out
for i in a b c; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 2>/dev/null | grep '^{' >> $out || exit 1
done
cat $out
bash scripts/gpu_prof.sh r5_base --steps 20 --warmup 5 | head -12
bash scripts/gpu_gemm.sh
