#!/bin/bash
# VERDICT r2 items 7 + 8: generation chars/s (3 precisions x 32/256/4096 names) and the fp64-oracle
# name identity across seeds / presets
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python bench/bench_generate.py --names 32,256,4096 \
  --modes engine,engine_fp32,engine_fp32_batched,engine_bf16x3,torch > gpurun_out/gen_speed.jsonl || exit 1
timeout -k 10 400 python scripts/gen_default_decision.py > gpurun_out/gen_oracle.jsonl || exit 1
echo done
