#!/bin/bash
# wavefront kernel probe + kernel/engine tests, then same-box A/B of the headline (new vs ab_old build)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 120 python scripts/probe_seq2.py > gpurun_out/probe_seq2.json && cat gpurun_out/probe_seq2.json || exit 1
H=512 B=256 timeout -k 10 120 python scripts/probe_seq.py || exit 1
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_engine_gpu.py -k "fwd_seq2 or lr_schedule" > gpurun_out/k2.log 2>&1; rc=$?; tail -2 gpurun_out/k2.log; [ $rc -ne 0 ] && exit $rc
bash scripts/gpu_so_ab.sh 3
