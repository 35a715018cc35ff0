#!/bin/bash
# session 41: staggered vs one-vmcnt GEMM on the h2048 logits and h1024 dX shapes
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
GEMM_ONLY256=1 GEMM_SHAPES=h2048.logits,h1024.dX,h1024.Gi timeout -k 10 300 python -u scripts/bench_gemm.py > gpurun_out/s41_gemm.jsonl 2> gpurun_out/s41_gemm.err || exit 1
python3 -c "
import json
for l in open('gpurun_out/s41_gemm.jsonl'):
    d=json.loads(l); print(d['shape'], {k[:-7]:v for k,v in d.items() if k.endswith('tflops')}, max([v for k,v in d.items() if k.endswith('relerr')] or [0]))"
