#!/bin/bash
# fused step tail in data-parallel mode: world-1 equivalence tests + --rccl-self bench / trace
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
: timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_engine_gpu.py tests/test_multigpu.py \
  -k "rccl_world1 or one_graph_step or multi_step_graph or tail_p_table or error_word or sharded or twin" \
  > gpurun_out/dptail_tests.log 2>&1; rc=0; [ $rc -ne 0 ] && { grep -E "^E |FAIL" gpurun_out/dptail_tests.log | head -30; exit $rc; }
for r in 1 2; do
  timeout -k 10 120 python bench.py --steps 300 --warmup 50 2>/dev/null | python3 -c "import json,sys; d=json.load(sys.stdin); print('nocomm', d['ms_per_step'])" || exit 1
  timeout -k 10 120 python bench.py --steps 300 --warmup 50 --rccl-self 2>/dev/null | python3 -c "import json,sys; d=json.loads([l for l in sys.stdin if l.startswith('{')][-1]); print('rccl-self', d['ms_per_step'], d['config']['collectives'])" || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_rself_tail -o run -- \
  python3 bench.py --steps 12 --warmup 4 --rccl-self > gpurun_out/prof_rself_tail.log 2>&1 || true
python3 scripts/analyze_trace.py gpurun_out/prof_rself_tail/run_kernel_trace.csv --timeline | tee gpurun_out/prof_rself_tail/summary.txt
