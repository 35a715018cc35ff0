#!/bin/bash
# Round-end evidence, part 2: the headline in the driver's form (3x, alternating with the 1-rank RCCL
# data-parallel structure), the secondary configs, the torch comparators, generation, and kernel
# traces of the headline, the config-4 shard and config 5 (copied into profiles/ by hand).
# usage: gpu_benches.sh TAG
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=${1:-final}
out=gpurun_out/benches_$tag.jsonl; : > $out
run() {
  local t=$1; shift
  line=$(timeout -k 10 300 python bench.py "$@" 2>/dev/null | grep '^{') || { echo "run failed ($t)"; exit 1; }
  echo "{\"tag\": \"$t\", \"bench\": $line}" >> $out
  echo "$t -> $(echo $line | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["ms_per_step"], d["value"])')"
}
for i in 1 2 3; do
  run headline_$i
  run rccl_self_$i --rccl-self --steps 20 --warmup 5
done
run h1024_l2_shard --preset h1024_l2 --per-gpu-batch 128 --steps 20 --warmup 5
run h2048_b512 --preset h2048 --per-gpu-batch 512 --steps 8 --warmup 2
run h1024_l2_b1024 --preset h1024_l2 --per-gpu-batch 1024 --steps 8 --warmup 2
run torch_h512 --impl torch --steps 10 --warmup 3
run torch_h1024_l2_shard --impl torch --preset h1024_l2 --per-gpu-batch 128 --steps 5 --warmup 2
run torch_h2048_b512 --impl torch --preset h2048 --per-gpu-batch 512 --steps 3 --warmup 1
timeout -k 10 300 python bench/bench_generate.py --names 32,256,4096 --modes engine,engine_fp32 > gpurun_out/gen_$tag.jsonl 2>/dev/null || exit 1
cat gpurun_out/gen_$tag.jsonl
bash scripts/gpu_prof.sh ${tag}_h512 --steps 20 --warmup 5 | head -10 && \
bash scripts/gpu_prof.sh ${tag}_c4 --preset h1024_l2 --per-gpu-batch 128 --steps 5 --warmup 2 | head -14 && \
bash scripts/gpu_prof.sh ${tag}_c5 --preset h2048 --per-gpu-batch 512 --steps 4 --warmup 2 | head -14
