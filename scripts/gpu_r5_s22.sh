#!/bin/bash
# session 22: row sums as v_dot2 in the R segments
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread -k "gemm or wgrad or library or bench_shape" > gpurun_out/s22_tests.log 2>&1
rc=$?; tail -2 gpurun_out/s22_tests.log; [ $rc -ne 0 ] && exit $rc
GEMM_ONLY256=1 GEMM_SHAPES=h2048.dW_hh,h1024.dWih timeout -k 10 300 python -u scripts/bench_gemm.py > gpurun_out/s22_gemm.jsonl 2> gpurun_out/s22_gemm.err || exit 1
python3 -c "
import json
for l in open('gpurun_out/s22_gemm.jsonl'):
    d=json.loads(l); print(d['shape'], {k[:-7]:v for k,v in d.items() if k.endswith('tflops') and 'ms' not in k})"
out=gpurun_out/s22_benches.jsonl; : > $out
run() { tag=$1; shift; line=$(timeout -k 10 300 "$@" 2>/dev/null | grep '^{') || { echo "fail $tag"; exit 1; }; echo "{\"tag\": \"$tag\", \"b\": $line}" >> $out; echo "$tag $(echo $line | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["ms_per_step"], d.get("final_loss"))')"; }
run c5_auto python bench.py --preset h2048 --per-gpu-batch 512 --steps 6 --warmup 2
GK_WGRAD_GEMM=lib run c5_lib python bench.py --preset h2048 --per-gpu-batch 512 --steps 6 --warmup 2
run c5_auto_b python bench.py --preset h2048 --per-gpu-batch 512 --steps 6 --warmup 2
GK_WGRAD_GEMM=lib run c5_lib_b python bench.py --preset h2048 --per-gpu-batch 512 --steps 6 --warmup 2
run h512 python bench.py --steps 20 --warmup 5
