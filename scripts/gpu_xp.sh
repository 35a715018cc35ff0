#!/bin/bash
# layer-0 input projection inside the forward: tests, same-box A/B (GK_FWD_XP=1/0, also with the
# batch preparation in the tail), trace
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_engine_gpu.py -k "input_projection_in_kernel or grads_match_cpu or multi_step or table_free or fused_tail or tail_p" > gpurun_out/xp_tests.log 2>&1
rc=$?; tail -2 gpurun_out/xp_tests.log; [ $rc -ne 0 ] && { grep -E "^E |FAIL" gpurun_out/xp_tests.log | head -20; exit $rc; }
out=gpurun_out/xp_ab.jsonl; : > $out
for i in 1 2; do for cfg in "1 0" "0 0" "1 1"; do
  set -- $cfg
  line=$(GK_FWD_XP=$1 GK_TAIL_BATCH=$2 timeout -k 10 200 python bench.py --steps 300 --warmup 50 2>/dev/null | grep '^{') || { echo "bench failed"; exit 1; }
  echo "{\"GK_FWD_XP\": $1, \"GK_TAIL_BATCH\": $2, \"bench\": $line}" >> $out
  echo "XP=$1 TB=$2 -> $(echo $line | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["ms_per_step"], d["final_loss"])')"
done; done
bash scripts/gpu_prof.sh xp --steps 20 --warmup 4 | head -12
