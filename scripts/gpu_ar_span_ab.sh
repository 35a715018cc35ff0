#!/bin/bash
# h1024_l2 (128 sequences per GPU) data-parallel step on a 1-rank RCCL communicator: the top
# group's collective open across layer 0's persistent backward kernel (GK_AR_SPAN=1, default) vs
# joined before it (GK_AR_SPAN=0) vs no communicator; then a kernel trace of the span step.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for rep in 1 2 3; do
  for mode in nocomm span join; do
    case $mode in nocomm) args=""; env="GK_AR_SPAN=1";; span) args="--rccl-self"; env="GK_AR_SPAN=1";; join) args="--rccl-self"; env="GK_AR_SPAN=0";; esac
    line=$(env $env timeout -k 10 200 python bench.py --preset h1024_l2 --per-gpu-batch 128 --steps 30 --warmup 5 $args 2>/dev/null | grep '^{') || { echo "failed $mode"; exit 1; }
    echo "$mode $(echo $line | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["ms_per_step"], d["config"]["collectives"])')"
  done
done
for mode in span join; do
  v=1; [ $mode = join ] && v=0
  GK_AR_SPAN=$v timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_l2_$mode -o run -- python3 bench.py --preset h1024_l2 --per-gpu-batch 128 --steps 6 --warmup 3 --rccl-self > gpurun_out/prof_l2_$mode.log 2>&1
  rc=$?; echo "prof $mode rc=$rc"; [ $rc -gt 1 ] && exit $rc
  python3 scripts/analyze_trace.py gpurun_out/prof_l2_$mode/run_kernel_trace.csv --overlap --timeline > gpurun_out/prof_l2_$mode/summary.txt
  head -40 gpurun_out/prof_l2_$mode/summary.txt
done
exit 0
