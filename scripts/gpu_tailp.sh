#!/bin/bash
# fused tail with the next step's P table + batch: equivalence tests, timeline, bench
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_engine_gpu.py \
  -k "one_graph_step or multi_step_graph or tail_p_table or error_word or late_workgroups or carry_graph or rccl_world1 or lr_schedule" \
  > gpurun_out/tailp_tests.log 2>&1; rc=$?; tail -3 gpurun_out/tailp_tests.log; [ $rc -ne 0 ] && { grep -E "^E |FAIL" gpurun_out/tailp_tests.log | head -30; exit $rc; }
timeout -k 10 120 python scripts/probe_tail.py > gpurun_out/ptail.txt 2>&1 && grep -v amdgpu gpurun_out/ptail.txt || exit 1
for i in 1 2; do timeout -k 10 120 python bench.py --steps 300 --warmup 50 2>/dev/null || exit 1; done
GK_TAIL_P=0 timeout -k 10 120 python bench.py --steps 300 --warmup 50 2>/dev/null || exit 1
timeout -k 10 120 python bench.py --steps 300 --warmup 50 --rccl-self 2>/dev/null || exit 1
GK_AR_FC_EARLY=0 timeout -k 10 120 python bench.py --steps 300 --warmup 50 --rccl-self 2>/dev/null || exit 1
