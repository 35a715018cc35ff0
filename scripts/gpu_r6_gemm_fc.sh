cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
GEMM_ONLY256= GEMM_SPLITS2=8,16,64 GEMM_SHAPES=h2048.dW_fc timeout -k 10 600 python scripts/bench_gemm.py > gpurun_out/r6_gemm_dwfc.jsonl 2> gpurun_out/r6_gemm_fc.err; rc=$?
python3 -c "
import json
for l in open('gpurun_out/r6_gemm_dwfc.jsonl'):
    r=json.loads(l); print(r['shape'], {k:v for k,v in r.items() if k.endswith('_us') and (k.startswith('algo2') or k.startswith('torch') or k.startswith('algo4'))})
"
exit $rc
