#!/bin/bash
# session 8: generator v5 (v3 + direct logits up to 8 names + one-round flag loads); forward with two
# flag polls in flight (wave_wait_load_pipe): engine tests + same-box A/B against the previous build
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread -k "generator or names or trainer_grads or bench_shape or persistent" > gpurun_out/s8_tests.log 2>&1
rc=$?; tail -3 gpurun_out/s8_tests.log; [ $rc -ne 0 ] && exit $rc
out=gpurun_out/s8_gen_probe.jsonl; : > $out
for n in 1 8 64; do
  timeout -k 10 120 python scripts/probe_gen_persist.py $n >> $out 2>>gpurun_out/s8_probe.err || exit 1
done
cat $out
bash scripts/gpu_so_ab.sh 3 --steps 300 --warmup 30 --min-warmup 300
