#!/bin/bash
# driver-form (K=20, W=5) fused vs phased tail, 6 alternating pairs
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
out=gpurun_out/tail_ab3.jsonl; : > $out
for i in 1 2 3 4 5 6; do for t in 1 0; do
  line=$(GK_TAIL=$t timeout -k 10 200 python bench.py --steps 20 --warmup 5 2>/dev/null | grep '^{') || { echo "bench failed"; exit 1; }
  echo "{\"GK_TAIL\": $t, \"ms\": $(echo $line | python3 -c 'import json,sys; print(json.load(sys.stdin)["ms_per_step"])')}" >> $out
  tail -1 $out
done; done
