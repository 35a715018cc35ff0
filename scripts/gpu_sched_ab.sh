#!/bin/bash
# Schedule A/B on one box: engine tests once, then the headline bench under each env variant
# (GK_* switches read at graph capture).  Each run under its own limit; stops at a crash-type exit.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
run() {  # name, timeout, cmd...
  local name=$1 to=$2; shift 2
  echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c1-400
  if [ $rc -gt 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
[ -n "$TESTS" ] && run engine 300 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread
# VARIANTS: space-separated list of "name:ENV=v,ENV2=v"
for spec in $VARIANTS; do
  name=${spec%%:*}; envs=${spec#*:}
  run "ab_$name" 200 env ${envs//,/ } python bench.py --steps 100 --warmup 20 ${BENCH_ARGS}
done
