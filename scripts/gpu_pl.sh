#!/bin/bash
# table-free layer-0 forward: kernel + engine tests, then same-box A/B (GK_FWD_PL=1/0) and a trace
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "table_free" tests/test_engine_gpu.py > gpurun_out/pl_tests.log 2>&1
rc=$?; tail -3 gpurun_out/pl_tests.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|error" gpurun_out/pl_tests.log | head -30; exit $rc; }
out=gpurun_out/pl_ab.jsonl; : > $out
for i in 1 2; do for pl in 1 0; do
  line=$(GK_FWD_PL=$pl timeout -k 10 200 python bench.py --steps 300 --warmup 50 2>/dev/null | grep '^{') || { echo "bench failed"; exit 1; }
  echo "{\"GK_FWD_PL\": $pl, \"bench\": $line}" >> $out
  echo "PL=$pl -> $(echo $line | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["ms_per_step"])')"
done; done
bash scripts/gpu_prof.sh pl --steps 20 --warmup 4 | head -12
