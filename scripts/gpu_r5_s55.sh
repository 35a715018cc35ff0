#!/bin/bash
# session 55: 128-row forward step tile on 8 waves (fwd64=2: 4-deep ring, 3: 3-deep) vs the 64-row
# default -- kernel tests, config-5 shard alternating, per-kernel trace of each
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "fwd_step" > gpurun_out/s55_tests.log 2>&1
rc=$?; tail -2 gpurun_out/s55_tests.log; [ $rc -ne 0 ] && exit $rc
out=gpurun_out/s55_benches.jsonl; : > $out
run() { tag=$1; shift; line=$(timeout -k 10 300 "$@" 2>/dev/null | grep '^{') || { echo "fail $tag"; exit 1; }; echo "{\"tag\": \"$tag\", \"b\": $line}" >> $out; echo "$tag $(echo $line | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["ms_per_step"], d.get("final_loss"))')"; }
for i in 1 2; do
  run c5_fwd64 python bench.py --preset h2048 --per-gpu-batch 512 --steps 6 --warmup 2
  run c5_w8ns4 python bench.py --preset h2048 --per-gpu-batch 512 --steps 6 --warmup 2 --variant fwd64=2
  run c5_w8ns3 python bench.py --preset h2048 --per-gpu-batch 512 --steps 6 --warmup 2 --variant fwd64=3
done
for v in 1 2 3; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/s55_prof$v -o run -- python3 bench.py --preset h2048 --per-gpu-batch 512 --steps 2 --warmup 1 --graph-steps 1 --variant fwd64=$v > gpurun_out/s55_prof$v.log 2>&1 || exit 1
  python3 scripts/analyze_trace.py gpurun_out/s55_prof$v/run_kernel_trace.csv --prologue > gpurun_out/s55_prof$v/summary.txt
  echo "== fwd64=$v"; head -4 gpurun_out/s55_prof$v/summary.txt
done
