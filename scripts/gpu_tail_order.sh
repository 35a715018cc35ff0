#!/bin/bash
# tail item ordering A/B (dW_fc / Adam blocks waiting for the dP chain) + P GEMM alone (GK_TAIL_BATCH=1 trace)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for r in 1 2; do
  for e in GK_TAIL_FC_WAIT=0 GK_TAIL_FC_WAIT=1 GK_TAIL_ADAM_WAIT=1; do
    env $e timeout -k 10 100 python bench.py --steps 300 --warmup 50 2>/dev/null | \
      python3 -c "import json,sys; d=json.load(sys.stdin); print('$e', d['ms_per_step'])" || exit 1
  done
done
GK_TAIL_FC_WAIT=1 timeout -k 10 100 python scripts/probe_tail.py > gpurun_out/ptail_fcwait.txt 2>&1 && grep -v amdgpu gpurun_out/ptail_fcwait.txt
export GK_TAIL_BATCH=1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_tb -o run -- python3 bench.py --steps 12 --warmup 4 > gpurun_out/prof_tb.log 2>&1
python3 scripts/analyze_trace.py gpurun_out/prof_tb/run_kernel_trace.csv --all | head -12
