#!/bin/bash
# driver-form bench (K=20, W=5): plan with groups up to 32 (1 single + 19) vs 2 singles + 9 vs G=10
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_engine_gpu.py -k "multi_step" > gpurun_out/plan_tests.log 2>&1
rc=$?; tail -2 gpurun_out/plan_tests.log; [ $rc -ne 0 ] && { grep -E "^E |FAIL" gpurun_out/plan_tests.log | head; exit $rc; }
out=gpurun_out/plan_ab2.jsonl; : > $out
for i in 1 2 3 4 5 6; do for g in 0 10; do
  line=$(timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --graph-steps $g 2>/dev/null | grep '^{') || { echo "bench failed"; exit 1; }
  echo "{\"graph_steps_arg\": $g, \"ms\": $(echo $line | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["ms_per_step"], ", \"G\": ", d["graph_steps"], ", \"lead\": ", d["lead_single_steps"])')}" >> $out
  tail -1 $out
done; done
