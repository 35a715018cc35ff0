#!/bin/bash
# adam_cast staging-tile pitch 66: tests touching the optimiser copies, trace, LDS-conflict counters
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_engine_gpu.py tests/test_kernels_gpu.py -k "phased or cast or adam or grads_match_cpu or multi_step or tail" > gpurun_out/adam_tests.log 2>&1
rc=$?; tail -2 gpurun_out/adam_tests.log; [ $rc -ne 0 ] && { grep -E "^E |FAIL" gpurun_out/adam_tests.log | head -20; exit $rc; }
for i in 1 2 3; do timeout -k 10 200 python bench.py --steps 300 --warmup 50 2>/dev/null | grep '^{' | python3 -c 'import json,sys; print("K=300", json.load(sys.stdin)["ms_per_step"])'; done
bash scripts/gpu_prof.sh adam66 --steps 20 --warmup 4 | head -10
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES --output-format csv -d gpurun_out/pmc_adam66 -o run -- python3 bench.py --steps 3 --warmup 2 > gpurun_out/pmc_adam66.log 2>&1
python3 - <<'PY'
import csv, glob, collections
f = glob.glob("gpurun_out/pmc_adam66/**/run_counter_collection.csv", recursive=True)
if not f: print("no counter csv"); raise SystemExit
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(f[0])):
    if "adam_cast" in r["Kernel_Name"] or "gru_bwd" in r["Kernel_Name"]:
        acc[r["Kernel_Name"][:40]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in acc.items():
    c, a = v.get("SQ_LDS_BANK_CONFLICT", 0), v.get("SQ_LDS_IDX_ACTIVE", 1)
    print(f"{k}: LDS conflict {100 * c / max(a, 1):.1f}%  insts {v.get('SQ_INSTS_LDS', 0):.0f}")
PY
