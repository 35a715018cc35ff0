#!/bin/bash
# session 9: poll sleep 1 (tree) vs 4 (ab_old) same-box A/B, headline and config-4 shard; persistent vs
# bf16-graph generation per char at 8-64 names (the bf16 mode's persistent cap)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
bash scripts/gpu_so_ab.sh 3 --steps 300 --warmup 30 --min-warmup 300 > gpurun_out/s9_ab_h512.txt 2>&1 || exit 1
cat gpurun_out/s9_ab_h512.txt
bash scripts/gpu_so_ab.sh 2 --preset h1024_l2 --per-gpu-batch 128 --steps 40 --warmup 10 --min-warmup 30 > gpurun_out/s9_ab_c4.txt 2>&1 || exit 1
cat gpurun_out/s9_ab_c4.txt
timeout -k 10 300 python scripts/gen_persist_vs_graph.py > gpurun_out/s9_gen_vs_graph.jsonl 2> gpurun_out/s9_gen.err || exit 1
cat gpurun_out/s9_gen_vs_graph.jsonl
