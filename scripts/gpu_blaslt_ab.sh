#!/bin/bash
# hipBLASLt path: kernel tests, engine test, then same-box A/B (GK_BLASLT=0 vs default) of the
# large-H presets (full preset batch on one GPU, and the per-GPU shard of the dp8 config).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm_library or gemm_nt" \
  tests/test_engine_gpu.py::test_trainer_grads_lds_step_kernels > gpurun_out/blaslt_tests.log 2>&1
rc=$?; tail -3 gpurun_out/blaslt_tests.log; [ $rc -ne 0 ] && exit $rc
run() {  # tag, args...
  local tag=$1; shift
  for v in 0 1; do
    GK_BLASLT=$v timeout -k 10 200 python bench.py "$@" > gpurun_out/blab_${tag}_$v.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { tail -5 gpurun_out/blab_${tag}_$v.log; exit $rc; }
    echo "$tag blaslt=$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/blab_${tag}_$v.log)"
  done
}
run h2048 --preset h2048 --steps 20 --warmup 5
run h2048_b512 --preset h2048 --per-gpu-batch 512 --steps 40 --warmup 5
run h1024_l2 --preset h1024_l2 --steps 40 --warmup 5
run h1024_l2_b128 --preset h1024_l2 --per-gpu-batch 128 --steps 100 --warmup 10
