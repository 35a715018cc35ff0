cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -m gpu -k "onehot" > gpurun_out/r6_onehot_tests.log 2>&1 || { tail -40 gpurun_out/r6_onehot_tests.log; exit 1; }
tail -2 gpurun_out/r6_onehot_tests.log
timeout -k 10 300 python scripts/probe_onehot.py | tee -a gpurun_out/r6_onehot_probe.jsonl && \
bash scripts/gpu_variant_ab.sh "gemm.onehot=0 gemm.onehot=1" 2 gpurun_out/r6_onehot_c5_ab.jsonl --preset h2048 --per-gpu-batch 512 --steps 8 --warmup 2 && \
bash scripts/gpu_prof.sh r6_c5_onehot --preset h2048 --per-gpu-batch 512 | head -8
