cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
bash scripts/gpu_prof.sh r6_c5_dwfc16 --preset h2048 --per-gpu-batch 512 | head -14 && \
timeout -k 10 300 python bench.py --preset h1024_l2 --per-gpu-batch 128 --steps 20 --warmup 5 | tail -1
