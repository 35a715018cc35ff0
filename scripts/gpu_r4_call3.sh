#!/bin/bash
# round 4: large-H persistent forward + backward first, then dW_fc in the embedding-side launch
# (tests + A/B) and the headline vs the round-3 build
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
bash scripts/gpu_r4_big.sh || exit 1
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 200 --timeout-method thread -k "dwfc or bench_shape" > gpurun_out/r4_c3_tests.log 2>&1
rc=$?; tail -6 gpurun_out/r4_c3_tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  for v in 1 0; do
    line=$(timeout -k 10 300 python bench.py --steps 20 --warmup 5 --variant dwfc_group=$v 2>/dev/null | grep '^{') || { echo "bench failed ($v)"; exit 1; }
    echo "{\"dwfc_group\": $v, \"round\": $i, \"bench\": $line}" >> gpurun_out/r4_dwfc_ab.jsonl
    echo "dwfc_group=$v $i $(echo $line | python3 -c 'import json,sys; print(json.load(sys.stdin)["ms_per_step"])')"
  done
done
bash scripts/gpu_multi_ab.sh "new ab_r3" 3 gpurun_out/r4_ab2_driver.jsonl --steps 20 --warmup 5 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r4_h512c -o run -- python3 bench.py --steps 10 --warmup 3 --min-warmup 50 > gpurun_out/prof_r4_h512c.log 2>&1 || exit 1
python3 scripts/analyze_trace.py gpurun_out/prof_r4_h512c/run_kernel_trace.csv > gpurun_out/prof_r4_h512c/summary.txt
cat gpurun_out/prof_r4_h512c/summary.txt
