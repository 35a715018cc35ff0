#!/bin/bash
# P table as split-K slabs summed by the forward gather: grads vs fp64, step equivalences, A/B bench
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_engine_gpu.py \
  -k "grads_match_cpu or one_graph_step or multi_step_graph or tail_p_table or rccl_world1 or odd_shapes or deterministic" \
  > gpurun_out/pslabs_tests.log 2>&1; rc=$?; tail -2 gpurun_out/pslabs_tests.log; [ $rc -ne 0 ] && { grep -E "^E |FAIL" gpurun_out/pslabs_tests.log | head -20; exit $rc; }
for r in 1 2 3; do
  for e in GK_P_SLABS=4 GK_P_SLABS=1; do
    env $e timeout -k 10 100 python bench.py --steps 300 --warmup 50 2>/dev/null | \
      python3 -c "import json,sys; d=json.load(sys.stdin); print('$e', d['ms_per_step'])" || exit 1
  done
done
