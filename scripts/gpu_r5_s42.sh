#!/bin/bash
# session 42: every 16x16-form gemm256 product on the staggered kernel -- GEMM/engine tests, benches
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/s42_tests.log 2>&1
rc=$?; tail -1 gpurun_out/s42_tests.log; [ $rc -ne 0 ] && exit $rc
out=gpurun_out/s42_benches.jsonl; : > $out
run() { tag=$1; shift; line=$(timeout -k 10 300 "$@" 2>/dev/null | grep '^{') || { echo "fail $tag"; exit 1; }; echo "{\"tag\": \"$tag\", \"b\": $line}" >> $out; echo "$tag $(echo $line | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["ms_per_step"], d.get("final_loss"))')"; }
run c5 python bench.py --preset h2048 --per-gpu-batch 512 --steps 6 --warmup 2
GK_GEMM256_PHASED=0 run c5_oldplain python bench.py --preset h2048 --per-gpu-batch 512 --steps 6 --warmup 2
run c4 python bench.py --preset h1024_l2 --per-gpu-batch 128 --steps 20 --warmup 5
run h512 python bench.py --steps 20 --warmup 5
run c5_b python bench.py --preset h2048 --per-gpu-batch 512 --steps 6 --warmup 2
