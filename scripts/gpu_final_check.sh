#!/bin/bash
# Final tree: the GPU suite + smoke, then config-5 / headline benches and the config-5 trace
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
bash scripts/gpu_round_final.sh || exit 1
: > gpurun_out/final2.jsonl
for i in 1 2; do
  timeout -k 10 300 python bench.py --preset h2048 --per-gpu-batch 512 --steps 8 --warmup 2 2>/dev/null | grep '^{' >> gpurun_out/final2.jsonl || exit 1
  timeout -k 10 300 python bench.py 2>/dev/null | grep '^{' >> gpurun_out/final2.jsonl || exit 1
done
python3 -c "import json; [print(json.loads(l)['config']['model'], json.loads(l)['ms_per_step']) for l in open('gpurun_out/final2.jsonl')]"
bash scripts/gpu_prof.sh final2_c5 --preset h2048 --per-gpu-batch 512 --steps 4 --warmup 2 | head -12
