#!/bin/bash
# session 53: gemm256 grouped raster A/B (GK_GEMM256_GROUPM 4 / 8 / 16 / 2, then 4 again), two passes
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for p in 1 2; do
  GEMM_ONLY256=1 GEMM_SHAPES=h2048.dW_hh,h1024.dWih,sq8192,sq4096,h2048.dH,h1024.Gi timeout -k 10 300 python -u scripts/bench_gemm.py > gpurun_out/s53_gemm_p$p.jsonl 2> gpurun_out/s53_gemm_p$p.err || exit 1
done
python3 - <<'PY'
import json
for p in (1, 2):
    for l in open(f"gpurun_out/s53_gemm_p{p}.jsonl"):
        d = json.loads(l); print(p, d["shape"], {k[:-7]: v for k, v in d.items() if k.endswith("tflops")})
PY
