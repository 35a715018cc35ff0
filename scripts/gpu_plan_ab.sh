#!/bin/bash
# driver-form bench (K=20, W=5): launch plan (2 singles + 2 groups of 9) vs plain groups of 10 / 4
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
out=gpurun_out/plan_ab.jsonl; : > $out
for i in 1 2 3 4 5; do for g in 0 10 4; do
  line=$(timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --graph-steps $g 2>/dev/null | grep '^{') || { echo "bench failed"; exit 1; }
  echo "{\"graph_steps_arg\": $g, \"ms\": $(echo $line | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["ms_per_step"], ", \"G\": ", d["graph_steps"], ", \"lead\": ", d["lead_single_steps"])')}" >> $out
  tail -1 $out
done; done
