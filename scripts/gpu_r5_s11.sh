#!/bin/bash
# session 11: 16-row persistent forward (gru_fwd_seq16): engine tests, then same-box A/B vs the 32-row kernel
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread -k "fwd16 or trainer_grads_match_cpu or exchange_ring or bench_shape or dp_pipelined or carry" > gpurun_out/s11_tests.log 2>&1
rc=$?; tail -3 gpurun_out/s11_tests.log; [ $rc -ne 0 ] && exit $rc
out=gpurun_out/s11_ab.jsonl; : > $out
for i in 1 2 3; do
  for v in 1 0; do
    line=$(timeout -k 10 200 python bench.py --steps 300 --warmup 30 --variant fwd16=$v 2>/dev/null | grep '^{') || exit 1
    echo "{\"fwd16\": $v, \"b\": $line}" >> $out
    echo "fwd16=$v $(echo $line | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["ms_per_step"], d["config"]["plan"])')"
  done
done
