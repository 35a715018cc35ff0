cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
bash scripts/gpu_pmc.sh r6_h512 && bash scripts/gpu_pmc.sh r6_c5 --preset h2048 --per-gpu-batch 512
