cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 200 --timeout-method thread -m gpu -k "big_backward_fused_dy or big_persistent_backward" > gpurun_out/r6_bigdy_tests.log 2>&1 || { tail -40 gpurun_out/r6_bigdy_tests.log; exit 1; }
tail -3 gpurun_out/r6_bigdy_tests.log
bash scripts/gpu_variant_ab.sh "big_dy=0 big_dy=1" 2 gpurun_out/r6_bigdy_c5_ab.jsonl --preset h2048 --per-gpu-batch 512 --steps 8 --warmup 2 && \
bash scripts/gpu_prof.sh r6_c5_bigdy --preset h2048 --per-gpu-batch 512 | head -14
