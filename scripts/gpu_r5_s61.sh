#!/bin/bash
# session 61: the dW_ih0 / dEmb / dW_fc group launch on 128-deep chunks (GK_SMALL_GROUP_DEPTH=2: 32 KB
# of LDS, every workgroup resident) vs 256-deep (default) -- tests under both, headline alternating, traces
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for ks in 2 0; do
  GK_SMALL_GROUP_DEPTH=$ks timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread -k "bench_shape or dwfc_in_embedding" > gpurun_out/s61_tests$ks.log 2>&1
  rc=$?; tail -1 gpurun_out/s61_tests$ks.log; [ $rc -ne 0 ] && exit $rc
done
out=gpurun_out/s61_benches.jsonl; : > $out
run() { tag=$1; shift; line=$(timeout -k 10 300 "$@" 2>/dev/null | grep '^{') || { echo "fail $tag"; exit 1; }; echo "{\"tag\": \"$tag\", \"b\": $line}" >> $out; echo "$tag $(echo $line | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["ms_per_step"], d.get("final_loss"))')"; }
for i in 1 2 3; do
  GK_SMALL_GROUP_DEPTH=2 run h512_d2 python bench.py --steps 20 --warmup 5
  run h512_d4 python bench.py --steps 20 --warmup 5
done
for ks in 2 0; do
  GK_SMALL_GROUP_DEPTH=$ks timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/s61_prof$ks -o run -- python3 bench.py --steps 3 --warmup 1 --graph-steps 1 > gpurun_out/s61_prof$ks.log 2>&1 || exit 1
  python3 scripts/analyze_trace.py gpurun_out/s61_prof$ks/run_kernel_trace.csv --prologue > gpurun_out/s61_prof$ks/summary.txt
  echo "== kslice $ks"; grep -v "prep" gpurun_out/s61_prof$ks/summary.txt | head -8
done
