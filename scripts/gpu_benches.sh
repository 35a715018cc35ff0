#!/bin/bash
# The secondary configs and the headline, one JSON line each (gpurun_out/benches.jsonl), plus kernel
# traces of the headline and the config-4 shard (profiles/ copies are made by hand).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
out=gpurun_out/benches.jsonl; : > $out
run() {
  local tag=$1; shift
  line=$(timeout -k 10 300 python bench.py "$@" 2>/dev/null | grep '^{') || { echo "run failed ($tag)"; exit 1; }
  echo "{\"tag\": \"$tag\", \"bench\": $line}" >> $out
  echo "$tag -> $(echo $line | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["ms_per_step"], d["value"])')"
}
run default_a
run default_b
run default_c
run h512_200 --steps 200 --warmup 20
run h1024_l2_shard --preset h1024_l2 --per-gpu-batch 128 --steps 50 --warmup 10
run h1024_l2_b1024 --preset h1024_l2 --per-gpu-batch 1024 --steps 10 --warmup 3
run h2048_b512 --preset h2048 --per-gpu-batch 512 --steps 6 --warmup 2
run rccl_self --rccl-self --steps 20 --warmup 5
timeout -k 10 300 python bench/bench_generate.py --names 32,256,4096 --modes engine,engine_fp32 > gpurun_out/gen.jsonl 2>/dev/null || exit 1
cat gpurun_out/gen.jsonl
bash scripts/gpu_prof.sh r4_h512_final --steps 20 --warmup 5 | head -10
bash scripts/gpu_prof.sh r4_c4_final --preset h1024_l2 --per-gpu-batch 128 --steps 5 --warmup 2 | head -14
