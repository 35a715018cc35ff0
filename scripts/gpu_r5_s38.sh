#!/bin/bash
# session 38: large-H backward with non-temporal exchange loads (GK_BIG_XNT) -- tests, config-5 A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
GK_BIG_XNT=1 timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread -k "big or h2048 or wgrad" > gpurun_out/s38_tests.log 2>&1
rc=$?; tail -1 gpurun_out/s38_tests.log; [ $rc -ne 0 ] && exit $rc
out=gpurun_out/s38_benches.jsonl; : > $out
run() { tag=$1; shift; line=$(timeout -k 10 300 "$@" 2>/dev/null | grep '^{') || { echo "fail $tag"; exit 1; }; echo "{\"tag\": \"$tag\", \"b\": $line}" >> $out; echo "$tag $(echo $line | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["ms_per_step"], d.get("final_loss"))')"; }
for i in 1 2; do
  GK_BIG_XNT=1 run c5_nt python bench.py --preset h2048 --per-gpu-batch 512 --steps 6 --warmup 2
  GK_BIG_XNT=0 run c5_rt python bench.py --preset h2048 --per-gpu-batch 512 --steps 6 --warmup 2
done
GK_BIG_XNT=1 timeout -k 10 300 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/pmc_c5_nt/g1 -o run -- python3 bench.py --preset h2048 --per-gpu-batch 512 --steps 3 --warmup 2 --min-warmup 0 > gpurun_out/pmc_c5_nt.log 2>&1 || exit 1
python3 scripts/analyze_pmc.py gpurun_out/pmc_c5_nt 2>/dev/null | head -4
