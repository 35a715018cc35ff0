#!/bin/bash
# session 51: persistent fp32 vs bf16 per-char graph after the end-to-end changes (bf16-mode cap)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/gen_persist_vs_graph.py 8,16,32,40,48,56,64 > gpurun_out/s51_vs.jsonl 2> gpurun_out/s51_vs.err || exit 1
cat gpurun_out/s51_vs.jsonl
