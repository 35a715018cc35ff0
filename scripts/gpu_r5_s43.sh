#!/bin/bash
# session 43: one-hot dP on the staggered 256-row GEMM (GK_DP256) -- tests, config-5 A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread -k "onehot or big or h2048 or wgrad or oracle or odd_shapes or grads" > gpurun_out/s43_tests.log 2>&1
rc=$?; tail -1 gpurun_out/s43_tests.log; [ $rc -ne 0 ] && exit $rc
out=gpurun_out/s43_benches.jsonl; : > $out
run() { tag=$1; shift; line=$(timeout -k 10 300 "$@" 2>/dev/null | grep '^{') || { echo "fail $tag"; exit 1; }; echo "{\"tag\": \"$tag\", \"b\": $line}" >> $out; echo "$tag $(echo $line | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["ms_per_step"], d.get("final_loss"))')"; }
for i in 1 2; do
  GK_DP256=1 run c5_dp256 python bench.py --preset h2048 --per-gpu-batch 512 --steps 6 --warmup 2
  GK_DP256=0 run c5_dp128 python bench.py --preset h2048 --per-gpu-batch 512 --steps 6 --warmup 2
done
GK_DP256=1 run c4_dp256 python bench.py --preset h1024_l2 --per-gpu-batch 128 --steps 20 --warmup 5
GK_DP256=0 run c4_dp128 python bench.py --preset h1024_l2 --per-gpu-batch 128 --steps 20 --warmup 5
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_c5b -o run -- python3 bench.py --preset h2048 --per-gpu-batch 512 --steps 3 --warmup 1 --graph-steps 1 > gpurun_out/prof_c5b.log 2>&1 || exit 1
python3 scripts/analyze_trace.py gpurun_out/prof_c5b/run_kernel_trace.csv --prologue > gpurun_out/prof_c5b/summary.txt
head -12 gpurun_out/prof_c5b/summary.txt
