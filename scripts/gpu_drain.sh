#!/bin/bash
# publishing wave's follow-up work inside its drain: tests, same-box A/B (GK_DRAIN_OVERLAP=1/0), probes
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_engine_gpu.py tests/test_kernels_gpu.py -k "grads_match_cpu or multi_step or deterministic or seq or fused_tail" > gpurun_out/drain_tests.log 2>&1
rc=$?; tail -2 gpurun_out/drain_tests.log; [ $rc -ne 0 ] && { grep -E "^E |FAIL" gpurun_out/drain_tests.log | head -20; exit $rc; }
out=gpurun_out/drain_ab.jsonl; : > $out
for i in 1 2 3; do for d in 1 0; do
  line=$(GK_BWD_FUSED_IN_DRAIN=$d timeout -k 10 200 python bench.py --steps 300 --warmup 50 2>/dev/null | grep '^{') || { echo "bench failed"; exit 1; }
  echo "{\"GK_BWD_FUSED_IN_DRAIN\": $d, \"bench\": $line}" >> $out
  echo "D=$d -> $(echo $line | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["ms_per_step"], d["final_loss"])')"
done; done
bash scripts/gpu_prof.sh drain --steps 20 --warmup 4 | head -8
