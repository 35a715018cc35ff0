#!/bin/bash
# session 3: phased GEMM v3 (tests, bench), config-4 shard and config-5 shard with the hand dW_hh
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "gemm256" > gpurun_out/s3_tests.log 2>&1
rc=$?; tail -2 gpurun_out/s3_tests.log; [ $rc -ne 0 ] && exit $rc
GEMM_ONLY256=1 GEMM_SHAPES=h2048.dW_hh,sq8192,h1024.dWih,h512.dW_hh timeout -k 10 300 python -u scripts/bench_gemm.py > gpurun_out/gemm_bench_v3.jsonl 2> gpurun_out/gemm_bench.err || exit 1
python3 -c "
import json
for l in open('gpurun_out/gemm_bench_v3.jsonl'):
    d=json.loads(l); print(d['shape'], {k:v for k,v in d.items() if k.endswith('tflops') and 'ms' not in k})"
out=gpurun_out/s3_benches.jsonl; : > $out
run() { tag=$1; shift; line=$(timeout -k 10 300 "$@" 2>/dev/null | grep '^{') || { echo "fail $tag"; exit 1; }; echo "{\"tag\": \"$tag\", \"b\": $line}" >> $out; echo "$tag $(echo $line | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["ms_per_step"], d.get("final_loss"))')"; }
run c4 python bench.py --preset h1024_l2 --per-gpu-batch 128 --steps 20 --warmup 5
run c5_lib python bench.py --preset h2048 --per-gpu-batch 512 --steps 6 --warmup 2
GK_WGRAD_GEMM=256 run c5_hand python bench.py --preset h2048 --per-gpu-batch 512 --steps 6 --warmup 2
run c4_b python bench.py --preset h1024_l2 --per-gpu-batch 128 --steps 20 --warmup 5
run h512 python bench.py --steps 20 --warmup 5
