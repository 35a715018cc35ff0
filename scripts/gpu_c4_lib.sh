#!/bin/bash
# config-4 shard: weight-gradient / dX products on hipBLASLt vs the hand GEMMs (A/B, alternating)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
run() { local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --preset h1024_l2 --per-gpu-batch 128 --steps 30 --warmup 5 2>/dev/null | grep '^{' | python3 -c "import json,sys; d=json.load(sys.stdin); print(json.dumps({'tag':'$tag','ms':d['ms_per_step']}))" | tee -a gpurun_out/c4_lib_ab.jsonl; }
for i in 1 2; do
  run default GK_X=0 || exit 1
  run wgrad_lib GK_WGRAD_GEMM=lib || exit 1
  run wgrad_lib_blaslt20 GK_WGRAD_GEMM=lib GK_BLASLT=1 GK_BLASLT_MIN_GFLOP=20 || exit 1
  run blaslt20 GK_BLASLT=1 GK_BLASLT_MIN_GFLOP=20 || exit 1
done
