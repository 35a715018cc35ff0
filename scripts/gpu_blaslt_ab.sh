#!/bin/bash
# hipBLASLt path: kernel tests, engine test, then same-box A/B (GK_BLASLT=0 vs default) of the
# large-H presets and the headline.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm_library or gemm_nt" \
  tests/test_engine_gpu.py::test_trainer_grads_lds_step_kernels > gpurun_out/blaslt_tests.log 2>&1
rc=$?; tail -3 gpurun_out/blaslt_tests.log; [ $rc -ne 0 ] && exit $rc
for p in h2048 h1024_l2 h512; do
  for v in 0 1; do
    st=20; [ $p = h512 ] && st=200
    GK_BLASLT=$v timeout -k 10 200 python bench.py --preset $p --steps $st --warmup 5 > gpurun_out/blab_${p}_$v.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { tail -5 gpurun_out/blab_${p}_$v.log; exit $rc; }
    echo "$p blaslt=$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/blab_${p}_$v.log)"
  done
done
