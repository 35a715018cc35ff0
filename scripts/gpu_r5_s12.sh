#!/bin/bash
# session 12: fixed cost of the timed region in the driver's 20-step form
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/probe_launch_overhead.py > gpurun_out/s12_launch.jsonl 2> gpurun_out/s12_launch.err
rc=$?; cat gpurun_out/s12_launch.jsonl; tail -3 gpurun_out/s12_launch.err; exit $rc
