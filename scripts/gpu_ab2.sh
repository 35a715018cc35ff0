#!/bin/bash
# generic alternating A/B of env settings on the headline bench: gpu_ab2.sh "ENV=a" "ENV=b" [rounds]
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
A=$1; B=$2; R=${3:-3}
for r in $(seq $R); do
  for e in "$A" "$B"; do
    env $e timeout -k 10 100 python bench.py --steps 200 --warmup 20 2>/dev/null | \
      python3 -c "import json,sys; d=json.load(sys.stdin); print('$e', d['ms_per_step'], 'G=%d' % d['graph_steps'], 'loss=%s' % d['final_loss'])" || exit 1
  done
done
