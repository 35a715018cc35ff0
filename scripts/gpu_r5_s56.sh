#!/bin/bash
# session 56: fused Adam / bf16 refresh on 32-row tiles (GK_ADAM_ROWS=32) vs 64-row -- bitwise test,
# bench-shape test, headline and config-4 alternating, per-kernel traces
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread -k "adam_tile_rows or bench_shape or dwfc_in_embedding" > gpurun_out/s56_tests.log 2>&1
rc=$?; tail -2 gpurun_out/s56_tests.log; [ $rc -ne 0 ] && exit $rc
out=gpurun_out/s56_benches.jsonl; : > $out
run() { tag=$1; shift; line=$(timeout -k 10 300 "$@" 2>/dev/null | grep '^{') || { echo "fail $tag"; exit 1; }; echo "{\"tag\": \"$tag\", \"b\": $line}" >> $out; echo "$tag $(echo $line | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["ms_per_step"], d.get("final_loss"))')"; }
for i in 1 2 3; do
  run h512_r64 python bench.py --steps 20 --warmup 5
  GK_ADAM_ROWS=32 run h512_r32 python bench.py --steps 20 --warmup 5
done
for i in 1 2; do
  run c4_r64 python bench.py --preset h1024_l2 --per-gpu-batch 128 --steps 20 --warmup 5
  GK_ADAM_ROWS=32 run c4_r32 python bench.py --preset h1024_l2 --per-gpu-batch 128 --steps 20 --warmup 5
done
for r in 64 32; do
  GK_ADAM_ROWS=$r timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/s56_prof$r -o run -- python3 bench.py --steps 3 --warmup 1 --graph-steps 1 > gpurun_out/s56_prof$r.log 2>&1 || exit 1
  python3 scripts/analyze_trace.py gpurun_out/s56_prof$r/run_kernel_trace.csv --prologue > gpurun_out/s56_prof$r/summary.txt
  echo "== rows $r"; grep -i "adam\|span" gpurun_out/s56_prof$r/summary.txt
done
