#!/bin/bash
# session 48: generator launch cost (entry -> char 0, end-to-end per generate) at 1 / 8 / 32 / 64 names
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
out=gpurun_out/s48_gen_probe.jsonl; : > $out
for n in 1 8 32 64; do
  timeout -k 10 120 python scripts/probe_gen_persist.py $n >> $out 2>>gpurun_out/s48_probe.err || exit 1
done
python3 -c "
import json
for l in open('$out'):
    d=json.loads(l); print(d['N'], d['us_per_char'], d['end_to_end_us_per_generate'], d['end_to_end_us_per_char'], d['launch_us'])"
