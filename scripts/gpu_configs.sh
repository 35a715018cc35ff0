#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
run() { local tag=$1; shift; timeout -k 10 300 python bench.py "$@" > gpurun_out/cfg_$tag.log 2>&1; local rc=$?; echo "$tag rc=$rc"; tail -1 gpurun_out/cfg_$tag.log; [ $rc -gt 1 ] && exit $rc; return 0; }
run h1024_l2 --preset h1024_l2 --per-gpu-batch 128 --steps 10 --warmup 3
run h2048 --preset h2048 --per-gpu-batch 512 --steps 5 --warmup 2
run h512_torch --impl torch --steps 10 --warmup 3
run h1024_l2_torch --impl torch --preset h1024_l2 --per-gpu-batch 128 --steps 5 --warmup 2
run h2048_torch --impl torch --preset h2048 --per-gpu-batch 512 --steps 3 --warmup 1
