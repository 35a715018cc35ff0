#!/bin/bash
# config-4 shard: 16-row persistent backward -- tests, then shard benches with it on / off, trace
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 200 --timeout-method thread -k "bwd16 or grads_match_cpu" > gpurun_out/c4_tests.log 2>&1
rc=$?; tail -4 gpurun_out/c4_tests.log; [ $rc -ne 0 ] && exit $rc
out=gpurun_out/c4_ab.jsonl
b() { timeout -k 10 300 python bench.py --preset h1024_l2 --per-gpu-batch 128 --steps 50 --warmup 10 "$@" 2>/dev/null | grep '^{'; }
for i in 1 2 3; do
  for v in 1 0; do
    l=$(b --variant bwd16=$v) || exit 1; echo "{\"bwd16\": $v, \"bench\": $l}" >> $out
    echo "bwd16=$v $(echo $l | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["ms_per_step"], d["config"].get("plan"))')"
  done
done
bash scripts/gpu_prof.sh c4_bwd16 --preset h1024_l2 --per-gpu-batch 128 --steps 5 --warmup 2 | head -8
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread -k "rccl or sharded or world1" > gpurun_out/dp_tests.log 2>&1
rc=$?; tail -3 gpurun_out/dp_tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for f in "" "--rccl-self"; do
    l=$(timeout -k 10 300 python bench.py --steps 20 --warmup 5 $f 2>/dev/null | grep '^{') || exit 1
    echo "{\"form\": \"$f\", \"bench\": $l}" >> gpurun_out/dp_struct_ab.jsonl
    echo "[$f] $(echo $l | python3 -c 'import json,sys; print(json.load(sys.stdin)["ms_per_step"])')"
  done
done
bash scripts/gpu_prof.sh r4_rccl_self2 --rccl-self --steps 20 --warmup 5 | head -12
