#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 120 python scripts/probe_seq_bwd.py || exit 1
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_engine_gpu.py -k "bwd_seq or grads_match_cpu or carry or one_graph or deterministic" > gpurun_out/t.log 2>&1; rc=$?; tail -2 gpurun_out/t.log; [ $rc -ne 0 ] && exit $rc
bash scripts/gpu_so_ab.sh 4
