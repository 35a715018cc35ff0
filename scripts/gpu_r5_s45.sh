#!/bin/bash
# session 45: staggered GEMM without s_setprio (default) vs MFMA segments at priority 1 -- tests, sweep, configs
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread -k "gemm or wgrad or bench_shape" > gpurun_out/s45_tests.log 2>&1
rc=$?; tail -1 gpurun_out/s45_tests.log; [ $rc -ne 0 ] && exit $rc
GEMM_ONLY256=1 GEMM_SHAPES=sq8192,sq4096,h2048.dW_hh,h1024.dWih timeout -k 10 500 python -u scripts/bench_gemm.py > gpurun_out/s45_gemm.jsonl 2> gpurun_out/s45_gemm.err || exit 1
python3 -c "
import json
for l in open('gpurun_out/s45_gemm.jsonl'):
    d=json.loads(l); print(d['shape'], {k[:-7]:v for k,v in d.items() if k.endswith('tflops') and (k.startswith('algo5s') or k.startswith('algo5p') or k.startswith('torch'))})"
out=gpurun_out/s45_benches.jsonl; : > $out
run() { tag=$1; shift; line=$(timeout -k 10 300 "$@" 2>/dev/null | grep '^{') || { echo "fail $tag"; exit 1; }; echo "{\"tag\": \"$tag\", \"b\": $line}" >> $out; echo "$tag $(echo $line | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["ms_per_step"], d.get("final_loss"))')"; }
run c5 python bench.py --preset h2048 --per-gpu-batch 512 --steps 6 --warmup 2
GK_GEMM256_PRIO=0 run c5_prio python bench.py --preset h2048 --per-gpu-batch 512 --steps 6 --warmup 2
run c4 python bench.py --preset h1024_l2 --per-gpu-batch 128 --steps 20 --warmup 5
GK_GEMM256_PRIO=0 run c4_prio python bench.py --preset h1024_l2 --per-gpu-batch 128 --steps 20 --warmup 5
