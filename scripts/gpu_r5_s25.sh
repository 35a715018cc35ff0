#!/bin/bash
# session 25: dW_fc over many tokens on gemm256p (GK_FC256) -- engine tests, config-5 A/B, c5 trace
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread -k "wgrad or h2048 or odd_shapes or bench_shape" > gpurun_out/s25_tests.log 2>&1
rc=$?; tail -2 gpurun_out/s25_tests.log; [ $rc -ne 0 ] && exit $rc
out=gpurun_out/s25_benches.jsonl; : > $out
run() { tag=$1; shift; line=$(timeout -k 10 300 "$@" 2>/dev/null | grep '^{') || { echo "fail $tag"; exit 1; }; echo "{\"tag\": \"$tag\", \"b\": $line}" >> $out; echo "$tag $(echo $line | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["ms_per_step"], d.get("final_loss"))')"; }
run c5_fc256 python bench.py --preset h2048 --per-gpu-batch 512 --steps 6 --warmup 2
GK_FC256=0 run c5_fc128 python bench.py --preset h2048 --per-gpu-batch 512 --steps 6 --warmup 2
run c5_fc256_b python bench.py --preset h2048 --per-gpu-batch 512 --steps 6 --warmup 2
GK_FC256=0 run c5_fc128_b python bench.py --preset h2048 --per-gpu-batch 512 --steps 6 --warmup 2
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_c5 -o run -- python3 bench.py --preset h2048 --per-gpu-batch 512 --steps 3 --warmup 1 --graph-steps 1 > gpurun_out/prof_c5.log 2>&1 || exit 1
python3 scripts/analyze_trace.py gpurun_out/prof_c5/run_kernel_trace.csv --prologue > gpurun_out/prof_c5/summary.txt
head -24 gpurun_out/prof_c5/summary.txt
