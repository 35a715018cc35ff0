#!/bin/bash
# session 36: GEMM schedule by k-tile count -- GEMM tests, config-4/5 benches and final-tree traces
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread -k "gemm or wgrad or library or bench_shape" > gpurun_out/s36_tests.log 2>&1
rc=$?; tail -1 gpurun_out/s36_tests.log; [ $rc -ne 0 ] && exit $rc
out=gpurun_out/s36_benches.jsonl; : > $out
run() { tag=$1; shift; line=$(timeout -k 10 300 "$@" 2>/dev/null | grep '^{') || { echo "fail $tag"; exit 1; }; echo "{\"tag\": \"$tag\", \"b\": $line}" >> $out; echo "$tag $(echo $line | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["ms_per_step"], d.get("final_loss"))')"; }
run c4 python bench.py --preset h1024_l2 --per-gpu-batch 128 --steps 20 --warmup 5
run c5 python bench.py --preset h2048 --per-gpu-batch 512 --steps 6 --warmup 2
GK_WGRAD_GEMM=lib run c5_lib python bench.py --preset h2048 --per-gpu-batch 512 --steps 6 --warmup 2
run c4_b python bench.py --preset h1024_l2 --per-gpu-batch 128 --steps 20 --warmup 5
run c5_b python bench.py --preset h2048 --per-gpu-batch 512 --steps 6 --warmup 2
for c in c4 c5; do
  if [ $c = c4 ]; then args="--preset h1024_l2 --per-gpu-batch 128 --steps 5 --warmup 2 --graph-steps 1"; else args="--preset h2048 --per-gpu-batch 512 --steps 3 --warmup 1 --graph-steps 1"; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_$c -o run -- python3 bench.py $args > gpurun_out/prof_$c.log 2>&1 || exit 1
  python3 scripts/analyze_trace.py gpurun_out/prof_$c/run_kernel_trace.csv --prologue > gpurun_out/prof_$c/summary.txt
  head -14 gpurun_out/prof_$c/summary.txt
done
