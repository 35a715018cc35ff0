#!/bin/bash
# Large-H per-step path after the step-kernel variant changes: GPU suite, h2048 kernel trace,
# h1024_l2 full-batch (per-step kernels) A/B of the 8-wave forward.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/full_gpu.log 2>&1
rc=$?; tail -2 gpurun_out/full_gpu.log; [ $rc -ne 0 ] && exit $rc
bash scripts/gpu_prof.sh h2048 --preset h2048 --per-gpu-batch 512 --steps 3 --warmup 1 | head -16 || exit 1
out=gpurun_out/ab_h1024l2_b1024_fwd8.jsonl; : > $out
for i in 1 2; do
  for e in GK_FWD_LDS8=1 GK_FWD_LDS8=0; do
    line=$(env $e timeout -k 10 200 python bench.py --preset h1024_l2 --per-gpu-batch 1024 --steps 10 --warmup 3 2>/dev/null | grep '^{') || { echo "run failed ($e)"; exit 1; }
    echo "{\"env\": \"$e\", \"rep\": $i, \"bench\": $line}" >> $out
    echo "$e -> $(echo $line | python3 -c 'import json,sys; print(json.load(sys.stdin)["ms_per_step"])')"
  done
done
