#!/bin/bash
# round-3 checks: bitwise step-path equality, new fault-tolerance tests, tail timeline, A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 120 python scripts/debug_tail_eq.py 2>&1 | grep -v "version\|Hostname\|Librccl\|amdgpu" || exit 1
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "late_workgroups or rides_the_last or one_graph or rccl_world1 or error_word or multi_step" > gpurun_out/t4_tests.log 2>&1
rc=$?; tail -3 gpurun_out/t4_tests.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" gpurun_out/t4_tests.log | head; exit $rc; }
timeout -k 10 60 python scripts/probe_tail.py 30 2>&1 | grep -v amdgpu || exit 1
bash scripts/gpu_ab2.sh GK_TAIL_FC=1 GK_TAIL_FC=0 3
