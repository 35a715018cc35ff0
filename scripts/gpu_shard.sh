#!/bin/bash
# Sharded optimiser (ZeRO-1) on one GPU: engine tests on a 1-rank communicator, then the step cost
# of the data-parallel structures (--rccl-self) with and without --shard-optim at h512 and h2048.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread -k "sharded or rccl_world1" -s > gpurun_out/shard_tests.log 2>&1
rc=$?; tail -3 gpurun_out/shard_tests.log; [ $rc -ne 0 ] && exit $rc
out=gpurun_out/ab_shard.jsonl; : > $out
run() {  # tag, args...
  local tag=$1; shift
  line=$(timeout -k 10 200 python bench.py "$@" 2>/dev/null | grep '^{') || { echo "run failed ($tag)"; exit 1; }
  echo "{\"tag\": \"$tag\", \"bench\": $line}" >> $out
  echo "$tag -> $(echo $line | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["ms_per_step"], d["final_loss"])')"
}
for i in 1 2; do
  run h512_plain --steps 200 --warmup 20
  run h512_rccl_self --steps 200 --warmup 20 --rccl-self
  run h512_rccl_self_shard --steps 200 --warmup 20 --rccl-self --shard-optim
done
for i in 1 2; do
  run h2048_rccl_self --preset h2048 --per-gpu-batch 512 --steps 5 --warmup 2 --rccl-self
  run h2048_rccl_self_shard --preset h2048 --per-gpu-batch 512 --steps 5 --warmup 2 --rccl-self --shard-optim
done
