#!/bin/bash
# session 46: extended persistent-generator shapes (one name at H = 256 / 512, 12 names)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 120 --timeout-method thread -k "generator_persistent" > gpurun_out/s46_tests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR" gpurun_out/s46_tests.log | tail -20; tail -1 gpurun_out/s46_tests.log; exit $rc
