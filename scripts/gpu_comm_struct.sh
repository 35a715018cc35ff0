#!/bin/bash
# Cost of the data-parallel step structure at 1 GPU (1-rank RCCL communicator recorded in the graph)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
b() { local tag=$1; shift; timeout -k 10 200 python bench.py --steps 30 --warmup 5 "$@" > gpurun_out/cs_$tag.log 2>&1; rc=$?
      echo "$tag rc=$rc $(tail -1 gpurun_out/cs_$tag.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["config"].get("collectives"))' 2>/dev/null)"; [ $rc -gt 1 ] && exit $rc; return 0; }
b h512 
b h512_self --rccl-self
b l2 --preset h1024_l2 --per-gpu-batch 128
b l2_self_single --preset h1024_l2 --per-gpu-batch 128 --rccl-self --bucket-mb 256
b l2_self_overlap --preset h1024_l2 --per-gpu-batch 128 --rccl-self --bucket-mb 4
exit 0
