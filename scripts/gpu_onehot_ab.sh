#!/bin/bash
# one-hot dP GEMM raster A/B: kernel tests, then h2048 step alternating the two builds' .so
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread -k "onehot or trainer" > gpurun_out/onehot.log 2>&1
rc=$?; tail -2 gpurun_out/onehot.log; [ $rc -ne 0 ] && exit $rc
bash scripts/gpu_prof.sh h2048_oh --preset h2048 --per-gpu-batch 512 --steps 3 --warmup 1 | head -8 || exit 1
REPS=2 bash scripts/gpu_step_ab.sh h2048_oh base
