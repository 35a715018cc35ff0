#!/bin/bash
# usage: gpu_pmc.sh TAG [bench args...] -> gpurun_out/pmc_TAG/{g1,g2,g3}/ + pmc_TAG/summary.txt
# Hardware counters per kernel (MFMA busy, LDS bank conflicts, HBM bytes), one counter group per
# rocprofv3 run, --pmc combined with --kernel-trace only (never with sys/runtime traces).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=$1; shift
out=gpurun_out/pmc_$tag; mkdir -p $out
groups=("SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU_MFMA_MOPS_BF16"
        "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES"
        "TCC_BUBBLE_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"
        "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"
        "TCC_HIT_sum TCC_MISS_sum"
        "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS")
# HBM bytes from the raw TCC counters (the derived FETCH_SIZE / WRITE_SIZE expressions of
# `rocprofv3 --list-avail`, evaluated in analyze_pmc.py: one group fits the 4-TCC-counter limit)
i=0
for g in "${groups[@]}"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $g --output-format csv -d $out/g$i -o run -- python3 bench.py --steps 3 --warmup 2 "$@" > $out/g$i.log 2>&1
  rc=$?; echo "pmc group $i rc=$rc"; [ $rc -gt 1 ] && exit $rc
done
python3 scripts/analyze_pmc.py $out | tee $out/summary.txt
