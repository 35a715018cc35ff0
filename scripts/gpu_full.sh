#!/bin/bash
# Round-end style validation: the whole GPU suite, smoke, the default bench, the h1024_l2 wave A/B.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/full_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/full_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -5 gpurun_out/smoke.log; exit 1; }
echo smoke ok
timeout -k 10 300 python bench.py > gpurun_out/bench_default.log 2>&1 || { tail -5 gpurun_out/bench_default.log; exit 1; }
grep '^{' gpurun_out/bench_default.log
out=gpurun_out/ab_wave.jsonl; : > $out
for i in 1 2; do
  for e in GK_FWD_WAVE=1 GK_FWD_WAVE=0; do
    line=$(env $e timeout -k 10 180 python bench.py --preset h1024_l2 --per-gpu-batch 128 --steps 50 --warmup 10 2>/dev/null | grep '^{') || { echo "run failed ($e)"; exit 1; }
    echo "{\"env\": \"$e\", \"rep\": $i, \"bench\": $line}" >> $out
    echo "$e -> $(echo $line | python3 -c 'import json,sys; print(json.load(sys.stdin)["ms_per_step"])')"
  done
done
bash scripts/gpu_prof.sh wave_h1024l2 --preset h1024_l2 --per-gpu-batch 128
