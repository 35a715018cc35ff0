#!/bin/bash
# per-phase probes: persistent forward (flags vs tagged exchange), small-batch fp32 generation
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
out=gpurun_out/r5_probe.jsonl; : > $out
for tag in 0 1; do
  XR=4 TAG=$tag timeout -k 10 120 python scripts/probe_seq.py >> $out 2>gpurun_out/probe.err || exit 1
done
for n in 1 8 32 64; do
  timeout -k 10 120 python scripts/probe_gen_persist.py $n >> $out 2>>gpurun_out/probe.err || exit 1
done
cat $out
