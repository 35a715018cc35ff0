#!/bin/bash
# GPU-box iteration run: kernel + engine tests, probes, headline bench
# (each step under its own time limit; stops at the first crash-type exit).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
run() {  # name, timeout, cmd...
  local name=$1 to=$2; shift 2
  echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc"; tail -3 "gpurun_out/$name.log"
  if [ $rc -gt 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
run kernels 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread
run engine 300 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread
for p in ${PROBES:-probe_fc}; do run $p 120 python scripts/$p.py; done
run bench 200 python bench.py --steps 50 --warmup 10
run bench2 200 python bench.py --steps 50 --warmup 10
