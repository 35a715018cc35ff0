#!/bin/bash
# session 29: generator layer-1 phase stamps (kept in LDS, shader clock)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
out=gpurun_out/s31_gen_probe.jsonl; : > $out
for n in 1 8 16; do
  timeout -k 10 120 python scripts/probe_gen_persist.py $n >> $out 2>>gpurun_out/s31_probe.err || exit 1
done
python3 -c "
import json
for l in open('$out'):
    d=json.loads(l); print(d['N'], d['us_per_char'], d['sclk_ghz'], d['L1_phase_us'])"
