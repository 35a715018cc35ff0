cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/full_gpu_r4a.log 2>&1
rc=$?; tail -5 gpurun_out/full_gpu_r4a.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r4a.log 2>&1; rc=$?; tail -3 gpurun_out/smoke_r4a.log; exit $rc
