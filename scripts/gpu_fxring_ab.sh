#!/bin/bash
# forward exchange ring (fwd_xring=4) vs one slot per step (0, default): alternating benches
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
run() { local tag=$1; shift
  timeout -k 10 300 python bench.py "$@" 2>/dev/null | grep '^{' | python3 -c "import json,sys; d=json.load(sys.stdin); print(json.dumps({'tag':'$tag','ms':d['ms_per_step'],'loss':d.get('final_loss')}))" | tee -a gpurun_out/fxring_ab.jsonl; }
for i in 1 2 3; do
  run h512_f4 --variant fwd_xring=4 || exit 1
  run h512_f0 || exit 1
  run c4_f4 --preset h1024_l2 --per-gpu-batch 128 --steps 30 --warmup 5 --variant fwd_xring=4 || exit 1
  run c4_f0 --preset h1024_l2 --per-gpu-batch 128 --steps 30 --warmup 5 || exit 1
done
