#!/bin/bash
# ring depth 2 vs 4 at the headline; the 1-rank data-parallel structure cost (rccl-self vs no comm)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
run() { local tag=$1; shift
  timeout -k 10 300 python bench.py "$@" 2>/dev/null | grep '^{' | python3 -c "import json,sys; d=json.load(sys.stdin); print(json.dumps({'tag':'$tag','ms':d['ms_per_step'],'loss':d.get('final_loss')}))" | tee -a gpurun_out/xr2_ab.jsonl; }
for i in 1 2 3; do
  run h512_xr4 || exit 1
  run h512_xr2 --variant bwd_xring=2 --variant fwd_xring=2 || exit 1
  run rccl_self --rccl-self || exit 1
done
