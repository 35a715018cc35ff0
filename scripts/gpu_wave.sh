#!/bin/bash
# Two-layer wavefront forward: correctness tests, same-box A/B (GK_FWD_WAVE) on the dp8 shard of
# h1024_l2 (128 seq x 64 per GPU), and a kernel trace of the wavefront step.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_engine_gpu.py \
  -k "grads_match_cpu or carry_hidden or one_graph_step" > gpurun_out/wave_tests.log 2>&1
rc=$?; tail -3 gpurun_out/wave_tests.log; [ $rc -ne 0 ] && exit $rc
out=gpurun_out/ab_wave.jsonl; : > $out
for i in 1 2; do
  for e in GK_FWD_WAVE=1 GK_FWD_WAVE=0; do
    line=$(env $e timeout -k 10 180 python bench.py --preset h1024_l2 --per-gpu-batch 128 --steps 50 --warmup 10 2>/dev/null | grep '^{') || { echo "run failed ($e)"; exit 1; }
    echo "{\"env\": \"$e\", \"rep\": $i, \"bench\": $line}" >> $out
    echo "$e -> $(echo $line | python3 -c 'import json,sys; print(json.load(sys.stdin)["ms_per_step"])')"
  done
done
bash scripts/gpu_prof.sh wave_h1024l2 --preset h1024_l2 --per-gpu-batch 128
