#!/bin/bash
# session 4: per-CU streaming probe (wavefront questions), final-tree traces h512 / c4 / c5, h512 PMC
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 120 ./scripts/probe_l2_stream 64 > gpurun_out/s4_l2_stream.jsonl 2> gpurun_out/s4_l2_stream.err
rc=$?; cat gpurun_out/s4_l2_stream.jsonl; [ $rc -ne 0 ] && { cat gpurun_out/s4_l2_stream.err; exit $rc; }
timeout -k 10 120 ./scripts/probe_l2_stream 16 > gpurun_out/s4_l2_stream16.jsonl 2>> gpurun_out/s4_l2_stream.err || exit 1
bash scripts/gpu_prof.sh r5_h512 || exit 1
bash scripts/gpu_prof.sh r5_c4 --preset h1024_l2 --per-gpu-batch 128 || exit 1
bash scripts/gpu_prof.sh r5_c5 --preset h2048 --per-gpu-batch 512 --steps 4 --warmup 2 || exit 1
bash scripts/gpu_pmc.sh r5_h512 --min-warmup 0 || exit 1
