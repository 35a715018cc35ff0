cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread -m gpu -k "adam or reduce or cast or bench_shape or sharded or trainer_grads" > gpurun_out/r6_lds_tests.log 2>&1 || { tail -40 gpurun_out/r6_lds_tests.log; exit 1; }
tail -2 gpurun_out/r6_lds_tests.log
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES --output-format csv -d gpurun_out/pmc_r6_lds/g2 -o run -- python3 bench.py --steps 3 --warmup 2 > gpurun_out/pmc_r6_lds.log 2>&1; echo "pmc rc=$?"
python3 scripts/analyze_pmc.py gpurun_out/pmc_r6_lds 2>&1 | head -12
bash scripts/gpu_prof.sh r6_lds --steps 20 --warmup 5 | head -10
for i in 1 2; do timeout -k 10 300 python bench.py 2>/dev/null | grep '^{' | python3 -c 'import json,sys; print(json.load(sys.stdin)["ms_per_step"])'; done
