#!/bin/bash
# full GPU suite + smoke + default bench + headline kernel trace + PMC (round-3 evidence)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=${1:-r3full}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/${tag}_gpu.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error" gpurun_out/${tag}_gpu.log | head -20; exit $rc; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
timeout -k 10 200 python bench.py > gpurun_out/${tag}_bench.json 2>/dev/null && cat gpurun_out/${tag}_bench.json || exit 1
bash scripts/gpu_prof.sh $tag --steps 20 --warmup 4 || exit 1
bash scripts/gpu_pmc.sh $tag
