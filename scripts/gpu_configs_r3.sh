#!/bin/bash
# round-3 numbers for every BASELINE config on one GPU (bench.py JSON lines) -> gpurun_out/r3_configs.jsonl
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
out=gpurun_out/r3_configs.jsonl; : > $out
run() { timeout -k 10 300 python bench.py "$@" 2>/dev/null | grep '^{' | tail -1 >> $out || exit 1; tail -1 $out | cut -c1-160; }
run --steps 300 --warmup 50
run --steps 300 --warmup 50
run --steps 300 --warmup 50 --rccl-self
run --preset h1024_l2 --per-gpu-batch 128 --steps 60 --warmup 10 --min-warmup 40
run --preset h1024_l2 --steps 20 --warmup 5 --min-warmup 10
run --preset h2048 --per-gpu-batch 512 --steps 20 --warmup 5 --min-warmup 10
run --impl torch --steps 20 --warmup 5 --min-warmup 5
