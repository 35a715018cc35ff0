#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
bash scripts/gpu_multi_ab.sh "new ab_r3 ab_dyb" 3 gpurun_out/r4_ab1_driver.jsonl --steps 20 --warmup 5 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r4_h512b -o run -- python3 bench.py --steps 10 --warmup 3 --min-warmup 50 > gpurun_out/prof_r4_h512b.log 2>&1 || exit 1
python3 scripts/analyze_trace.py gpurun_out/prof_r4_h512b/run_kernel_trace.csv > gpurun_out/prof_r4_h512b/summary.txt
cat gpurun_out/prof_r4_h512b/summary.txt
GEMM_SHAPES=h512.dW_fc,h512.P,h512.dEmb,h512.dW_ih0 timeout -k 10 300 python scripts/bench_gemm.py > gpurun_out/r4_gemm_h512.jsonl 2>&1 || exit 1
python3 - <<'PY'
import json
for l in open("gpurun_out/r4_gemm_h512.jsonl"):
    if not l.startswith("{"): continue
    d = json.loads(l)
    print(d["shape"], {k[:-3]: v for k, v in d.items() if k.endswith("_us")})
PY
timeout -k 10 120 python scripts/probe_fc.py > gpurun_out/r4_probe_fc.txt 2>&1 || exit 1
cat gpurun_out/r4_probe_fc.txt
