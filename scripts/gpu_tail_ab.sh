#!/bin/bash
# fused-tail A/B: timeline probes and alternating 200-step benches (env knobs), phased tail baseline
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
bench() {  # label, env...
  local label=$1; shift
  env "$@" timeout -k 10 100 python bench.py --steps 200 --warmup 20 2>/dev/null | \
    python3 -c "import json,sys; d=json.load(sys.stdin); print('$label', d['ms_per_step'], 'G=%d' % d['graph_steps'])"
}
timeout -k 10 60 python scripts/probe_tail.py 30 2>&1 | grep -v amdgpu.ids || exit 1
GK_TAIL_ADAM_WAIT=1 timeout -k 10 60 python scripts/probe_tail.py 30 2>&1 | grep -v amdgpu.ids || exit 1
for r in 1 2; do
  bench "tail" GK_TAIL_ADAM_WAIT=0 || exit 1
  bench "tail+adamwait" GK_TAIL_ADAM_WAIT=1 || exit 1
  bench "phased-tail" GK_TAIL=0 || exit 1
done
