#!/bin/bash
# session 47: generation speed refresh on the final tree (reference model, 1 / 8 / 32 / 256 / 4096 names)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u bench/bench_generate.py --names 1,8,32,256,4096 --modes engine,engine_fp32,torch > gpurun_out/s47_gen.jsonl 2> gpurun_out/s47_gen.err || exit 1
python3 -c "
import json
for l in open('gpurun_out/s47_gen.jsonl'):
    d=json.loads(l); print(d['names'], {k: (v.get('chars_per_s'), v.get('us_per_char_step'), v.get('persistent')) for k, v in d.items() if isinstance(v, dict)})"
