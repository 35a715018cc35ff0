#!/bin/bash
# h1024_l2 (128 sequences per GPU) data-parallel step structure on a 1-rank communicator: no comm vs
# in-graph collectives forked on the comm stream vs in line on the step stream (GK_AR_FORK=0)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for rep in 1 2; do
  for mode in nocomm fork inline; do
    case $mode in nocomm) args=""; env="";; fork) args="--rccl-self"; env="";; inline) args="--rccl-self"; env="GK_AR_FORK=0";; esac
    line=$(env $env timeout -k 10 200 python bench.py --preset h1024_l2 --per-gpu-batch 128 --steps 20 --warmup 5 $args 2>/dev/null | grep '^{') || { echo "failed $mode"; exit 1; }
    echo "$mode $(echo $line | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["ms_per_step"], d["config"]["collectives"])')"
  done
done
