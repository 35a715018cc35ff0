#!/bin/bash
# h2048 weight-gradient engine A/B (gemm256 vs hipBLASLt) on the new default plan, then round-4 PMC
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread -k "big_persistent" > gpurun_out/r4_c6_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r4_c6_tests.log; [ $rc -ne 0 ] && exit $rc
out=gpurun_out/r4_h2048_wgrad_ab.jsonl
b() { timeout -k 10 300 python bench.py --preset h2048 --per-gpu-batch 512 --steps 6 --warmup 2 2>/dev/null | grep '^{'; }
for i in 1 2; do
  l=$(b) || exit 1; echo "{\"form\": \"default\", \"bench\": $l}" >> $out
  l=$(GK_WGRAD_GEMM=lib b) || exit 1; echo "{\"form\": \"GK_WGRAD_GEMM=lib\", \"bench\": $l}" >> $out
  l=$(GK_BLASLT=1 b) || exit 1; echo "{\"form\": \"GK_BLASLT=1\", \"bench\": $l}" >> $out
  l=$(GK_BLASLT=1 GK_WGRAD_GEMM=lib b) || exit 1; echo "{\"form\": \"GK_BLASLT=1 GK_WGRAD_GEMM=lib\", \"bench\": $l}" >> $out
done
python3 -c '
import json
for l in open("'$out'"):
    d = json.loads(l); print(d["form"], d["bench"]["ms_per_step"])'
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread -k "dwfc" > gpurun_out/r4_c6_tests2.log 2>&1
rc=$?; tail -3 gpurun_out/r4_c6_tests2.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  for v in 1 2; do
    line=$(timeout -k 10 300 python bench.py --steps 20 --warmup 5 --variant dwfc_group=$v 2>/dev/null | grep '^{') || { echo "bench failed ($v)"; exit 1; }
    echo "{\"dwfc_group\": $v, \"round\": $i, \"bench\": $line}" >> gpurun_out/r4_dwfc2_ab.jsonl
    echo "dwfc_group=$v $i $(echo $line | python3 -c 'import json,sys; print(json.load(sys.stdin)["ms_per_step"])')"
  done
done
bash scripts/gpu_r4_call4.sh
