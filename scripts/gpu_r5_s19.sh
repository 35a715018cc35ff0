#!/bin/bash
# session 19: staggered phased GEMM as the only phased form -- GEMM tests, full shape sweep, config-4/5
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "gemm" > gpurun_out/s19_tests.log 2>&1
rc=$?; tail -2 gpurun_out/s19_tests.log; [ $rc -ne 0 ] && exit $rc
GEMM_ONLY256=1 timeout -k 10 500 python -u scripts/bench_gemm.py > gpurun_out/s19_gemm.jsonl 2> gpurun_out/s19_gemm.err || exit 1
python3 -c "
import json
for l in open('gpurun_out/s19_gemm.jsonl'):
    d=json.loads(l); print(d['shape'], {k[:-7]:v for k,v in d.items() if k.endswith('tflops') and 'ms' not in k})"
out=gpurun_out/s19_benches.jsonl; : > $out
run() { tag=$1; shift; line=$(timeout -k 10 300 "$@" 2>/dev/null | grep '^{') || { echo "fail $tag"; exit 1; }; echo "{\"tag\": \"$tag\", \"b\": $line}" >> $out; echo "$tag $(echo $line | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["ms_per_step"], d.get("final_loss"))')"; }
run c5_lib python bench.py --preset h2048 --per-gpu-batch 512 --steps 6 --warmup 2
GK_WGRAD_GEMM=256 run c5_hand python bench.py --preset h2048 --per-gpu-batch 512 --steps 6 --warmup 2
run c4 python bench.py --preset h1024_l2 --per-gpu-batch 128 --steps 20 --warmup 5
GK_WGRAD_GEMM=256 run c5_hand_b python bench.py --preset h2048 --per-gpu-batch 512 --steps 6 --warmup 2
run c5_lib_b python bench.py --preset h2048 --per-gpu-batch 512 --steps 6 --warmup 2
run h512 python bench.py --steps 20 --warmup 5
