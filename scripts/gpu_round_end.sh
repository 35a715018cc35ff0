#!/bin/bash
# Round-end evidence on the current tree: GPU suite, smoke, default bench, 200-step headline, the
# secondary configs, and a headline kernel trace (profiles/).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/full_gpu.log 2>&1
rc=$?; tail -2 gpurun_out/full_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
out=gpurun_out/round_end_benches.jsonl; : > $out
run() {
  local tag=$1; shift
  line=$(timeout -k 10 300 python bench.py "$@" 2>/dev/null | grep '^{') || { echo "run failed ($tag)"; exit 1; }
  echo "{\"tag\": \"$tag\", \"bench\": $line}" >> $out
  echo "$tag -> $(echo $line | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["ms_per_step"], d["value"])')"
}
run default
run h512_200 --steps 200 --warmup 20
run h512_200b --steps 200 --warmup 20
run h1024_l2_shard --preset h1024_l2 --per-gpu-batch 128 --steps 50 --warmup 10
run h1024_l2_b1024 --preset h1024_l2 --per-gpu-batch 1024 --steps 10 --warmup 3
run h2048_b512 --preset h2048 --per-gpu-batch 512 --steps 6 --warmup 2
bash scripts/gpu_prof.sh h512_final --steps 20 --warmup 5 | head -12
