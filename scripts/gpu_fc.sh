#!/bin/bash
# forward FC pipeline: tests, same-box A/B (GK_FWD_FC=1/0), trace
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_engine_gpu.py -k "fc_pipeline or grads_match_cpu" > gpurun_out/fc_tests.log 2>&1
rc=$?; tail -3 gpurun_out/fc_tests.log; [ $rc -ne 0 ] && { grep -E "^E |FAIL|Error" gpurun_out/fc_tests.log | head -30; exit $rc; }
out=gpurun_out/fc_ab.jsonl; : > $out
for i in 1 2; do for fc in 1 0; do
  line=$(GK_FWD_FC=$fc timeout -k 10 200 python bench.py --steps 300 --warmup 50 2>/dev/null | grep '^{') || { echo "bench failed"; exit 1; }
  echo "{\"GK_FWD_FC\": $fc, \"bench\": $line}" >> $out
  echo "FC=$fc -> $(echo $line | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["ms_per_step"], d["final_loss"])')"
done; done
bash scripts/gpu_prof.sh fc --steps 20 --warmup 4 | head -12
