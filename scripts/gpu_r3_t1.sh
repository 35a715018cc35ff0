#!/bin/bash
# round-3 fused-tail check: smoke, the step-path GPU tests, tail timeline probe, bench, kernel trace
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=${1:-t1}
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1 || { cat gpurun_out/${tag}_smoke.log; exit 1; }
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 120 --timeout-method thread -k "one_graph or deterministic or adam_step or multi_step or error_word or persistent_spin or rccl_world1 or lr_schedule or grads_match_cpu" > gpurun_out/${tag}_tests.log 2>&1; rc=$?; tail -5 gpurun_out/${tag}_tests.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/${tag}_tests.log | head -20; exit $rc; }
timeout -k 10 60 python scripts/probe_tail.py 30 2>&1 | grep -v amdgpu.ids
timeout -k 10 200 python bench.py --steps 48 > gpurun_out/${tag}_bench.json 2>gpurun_out/${tag}_bench.err; cat gpurun_out/${tag}_bench.json
bash scripts/gpu_prof.sh $tag --steps 20 --warmup 4
