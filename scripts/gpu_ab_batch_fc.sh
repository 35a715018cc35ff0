#!/bin/bash
# A/B: next-step batch preparation inside the fused tail; --rccl-self traces with/without the early FC collective
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for r in 1 2; do
  for e in GK_TAIL_BATCH=1 GK_TAIL_BATCH=0; do
    env $e timeout -k 10 100 python bench.py --steps 300 --warmup 50 2>/dev/null | \
      python3 -c "import json,sys; d=json.load(sys.stdin); print('$e', d['ms_per_step'])" || exit 1
  done
done
for e in GK_AR_FC_EARLY=1 GK_AR_FC_EARLY=0; do
  export $e
  tag=rself_${e##*=}
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_$tag -o run -- \
    python3 bench.py --steps 12 --warmup 4 --rccl-self > gpurun_out/prof_$tag.log 2>&1 || true
  echo "== $e"
  python3 scripts/analyze_trace.py gpurun_out/prof_$tag/run_kernel_trace.csv --overlap --timeline > gpurun_out/prof_$tag/summary.txt 2>&1
  head -40 gpurun_out/prof_$tag/summary.txt
done
