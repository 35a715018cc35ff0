#!/bin/bash
# Round-5 start: headline bench x3 + kernel trace of the headline step; gemm256 phased checks;
# the pipelined DP tail (test + rccl-self A/B)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
out=gpurun_out/r5_base.jsonl; : > $out
for i in a b c; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 2>/dev/null | grep '^{' >> $out || exit 1
done
cat $out
bash scripts/gpu_prof.sh r5_base --steps 20 --warmup 5 | head -12
bash scripts/gpu_gemm.sh || exit 1
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -k "dp_pipelined or rccl_world1" -x -q --timeout 120 --timeout-method thread > gpurun_out/dp_test.log 2>&1
rc=$?; tail -3 gpurun_out/dp_test.log; [ $rc -ne 0 ] && exit $rc
out=gpurun_out/r5_dp.jsonl; : > $out
for i in a b; do
  for m in 1 0; do
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --rccl-self --dp-pipeline $m 2>/dev/null | grep '^{' >> $out || exit 1
  done
done
python3 -c "
import json
for l in open('$out'): d=json.loads(l); print(d['config']['dp_pipeline'], d['ms_per_step'], d['config']['collectives'])"
