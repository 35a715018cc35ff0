#!/bin/bash
# round-5 final tree: full GPU suite, smoke, headline (driver form) x2, config-4 / config-5 shards,
# generation speed table
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/final_suite.log 2>&1
rc=$?; tail -3 gpurun_out/final_suite.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final_smoke.log 2>&1
rc=$?; tail -2 gpurun_out/final_smoke.log; [ $rc -ne 0 ] && exit $rc
out=gpurun_out/final_benches.jsonl; : > $out
run() { tag=$1; shift; line=$(timeout -k 10 300 "$@" 2>/dev/null | grep '^{') || { echo "fail $tag"; exit 1; }; echo "{\"tag\": \"$tag\", \"b\": $line}" >> $out; echo "$tag $(echo $line | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["ms_per_step"], d.get("final_loss"))')"; }
run h512 python bench.py --steps 20 --warmup 5
run h512_b python bench.py --steps 20 --warmup 5
run c4 python bench.py --preset h1024_l2 --per-gpu-batch 128 --steps 20 --warmup 5
run c5 python bench.py --preset h2048 --per-gpu-batch 512 --steps 6 --warmup 2
timeout -k 10 300 python bench/bench_generate.py --names 1,8,64,256,4096 --modes engine,engine_fp32 > gpurun_out/final_generate.jsonl 2> gpurun_out/final_generate.err || exit 1
python3 - <<'PY'
import json
for l in open("gpurun_out/final_generate.jsonl"):
    if l.startswith("{"):
        d = json.loads(l); print({k: v for k, v in d.items() if not isinstance(v, (dict, list))})
PY
