cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
GEMM_SPLITS2=4,16,32 GEMM_SHAPES=h1024.dW_fc,h1024.dX,h1024.dW_hh,h1024.dWih timeout -k 10 600 python scripts/bench_gemm.py > gpurun_out/r6_gemm_c4.jsonl 2> gpurun_out/r6_gemm_fc.err; rc=$?
python3 -c "
import json
for l in open('gpurun_out/r6_gemm_c4.jsonl'):
    r=json.loads(l); print(r['shape'], r['splits'], {k:v for k,v in r.items() if k.endswith('_us')})
"
exit $rc
