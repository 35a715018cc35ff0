#!/bin/bash
# Round-5 session 1: correctness of this round's kernels first, then the A/B benches and traces
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread \
  -k "exchange_ring or dp_pipelined or rccl_world1 or gemm256 or bench_shape" > gpurun_out/r5_tests.log 2>&1
rc=$?; grep -E "passed|failed|error" gpurun_out/r5_tests.log | tail -3; [ $rc -ne 0 ] && exit $rc
out=gpurun_out/r5_base.jsonl; : > $out
for i in a b; do
  for v in 1 0; do
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --variant fwd_tag=$v 2>/dev/null | grep '^{' | sed "s/^{/{\"fwd_tag\": $v, /" >> $out || exit 1
  done
done
python3 -c "
import json
for l in open('$out'): d=json.loads(l); print('fwd_tag', d['fwd_tag'], d['ms_per_step'], d['final_loss'])"
out2=gpurun_out/r5_dp.jsonl; : > $out2
for m in 1 0; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --rccl-self --dp-pipeline $m 2>/dev/null | grep '^{' >> $out2 || exit 1
done
python3 -c "
import json
for l in open('$out2'): d=json.loads(l); print('dp_pipeline', d['config']['dp_pipeline'], d['ms_per_step'], d['config']['collectives'])"
bash scripts/gpu_prof.sh r5_base --steps 20 --warmup 5 | head -12
bash scripts/gpu_r5_probe.sh
GEMM_ONLY256=1 GEMM_SHAPES=h2048.dW_hh,sq8192,sq4096,h1024.dWih,h1024.Gi timeout -k 10 300 python -u scripts/bench_gemm.py > gpurun_out/gemm_bench.jsonl 2> gpurun_out/gemm_bench.err
cat gpurun_out/gemm_bench.jsonl
