#!/bin/bash
# multi-step graph size: tests (G up to 16) and the driver-form bench at G = 4 / 10 / 20-capped
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_engine_gpu.py -k "multi_step_graph" > gpurun_out/gs_tests.log 2>&1
rc=$?; tail -2 gpurun_out/gs_tests.log; [ $rc -ne 0 ] && { grep -E "^E |FAIL" gpurun_out/gs_tests.log | head; exit $rc; }
out=gpurun_out/gsteps_ab.jsonl; : > $out
for i in 1 2; do for g in 4 10 0; do
  line=$(timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --graph-steps $g 2>/dev/null | grep '^{') || { echo "bench failed"; exit 1; }
  echo "{\"graph_steps_arg\": $g, \"bench\": $line}" >> $out
  echo "G=$g -> $(echo $line | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["ms_per_step"], d["graph_steps"])')"
done; done
for g in 4 0; do
  line=$(timeout -k 10 200 python bench.py --steps 300 --warmup 50 --graph-steps $g 2>/dev/null | grep '^{') || exit 1
  echo "{\"graph_steps_arg\": $g, \"steps\": 300, \"bench\": $line}" >> $out
  echo "K=300 G=$g -> $(echo $line | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["ms_per_step"], d["graph_steps"])')"
done
