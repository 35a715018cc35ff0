#!/bin/bash
# GPU-box check: numerics tests, smoke, short bench.  Stops at the first crash-type exit
# (fault/abort/segv/timeout); plain test failures (rc 1) still let later steps run.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
step() {  # name, timeout, cmd...
  local name=$1 to=$2; shift 2
  echo "== $name" ; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc"; tail -5 "gpurun_out/$name.log"
  if [ $rc -gt 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
python -m gru_mpi_cuda_amd.build_ext > gpurun_out/build.log 2>&1 || { echo "BUILD FAILED"; tail -20 gpurun_out/build.log; exit 3; }
step kernels 500 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread
step engine 500 python -u -m pytest tests/test_engine_gpu.py tests/test_capi_gpu.py -x -q --timeout 120 --timeout-method thread
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
step bench 300 python bench.py --steps 20 --warmup 5
