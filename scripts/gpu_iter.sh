#!/bin/bash
# One build -> measure iteration on the GPU box: kernel + engine tests, a short bench, and a
# rocprofv3 kernel trace of the headline step.   usage: gpu_iter.sh TAG [bench args...]
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=$1; shift
run() {  # name, timeout, cmd...   (stops the script on a crash-type exit)
  local name=$1 to=$2; shift 2
  echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/${tag}_$name.log" 2>&1
  local rc=$?; echo "   rc=$rc"; tail -4 "gpurun_out/${tag}_$name.log"
  if [ $rc -gt 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
run tests 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py tests/test_capi_gpu.py -x -q --timeout 120 --timeout-method thread
run bench 300 python bench.py --steps 50 --warmup 10 "$@"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o run -- python3 bench.py --steps 10 --warmup 3 "$@" > gpurun_out/prof_$tag.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -gt 1 ] && exit $rc
python3 scripts/analyze_trace.py gpurun_out/prof_$tag/run_kernel_trace.csv | tee gpurun_out/prof_$tag/summary.txt
