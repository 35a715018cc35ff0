#!/bin/bash
# session 54: Adam of the early-complete tensors inside the embedding GEMM group -- bitwise test,
# bench-shape oracle test, headline A/B (alternating), kernel trace of the new default
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread -k "adam_in_group or bench_shape or dwfc_in_embedding or oracle" > gpurun_out/s54_tests.log 2>&1
rc=$?; tail -2 gpurun_out/s54_tests.log; [ $rc -ne 0 ] && exit $rc
out=gpurun_out/s54_benches.jsonl; : > $out
run() { tag=$1; shift; line=$(timeout -k 10 200 "$@" 2>/dev/null | grep '^{') || { echo "fail $tag"; exit 1; }; echo "{\"tag\": \"$tag\", \"b\": $line}" >> $out; echo "$tag $(echo $line | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["ms_per_step"], d.get("final_loss"))')"; }
for i in 1 2 3; do
  run h512_group python bench.py --steps 20 --warmup 5
  GK_OPT_IN_GROUP=0 run h512_sep python bench.py --steps 20 --warmup 5
done
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/s54_prof -o run -- python3 bench.py --steps 3 --warmup 1 --graph-steps 1 > gpurun_out/s54_prof.log 2>&1 || exit 1
python3 scripts/analyze_trace.py gpurun_out/s54_prof/run_kernel_trace.csv --prologue > gpurun_out/s54_prof/summary.txt
head -12 gpurun_out/s54_prof/summary.txt
