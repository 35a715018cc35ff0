#!/bin/bash
# usage: gpu_probe_pmc.sh TAG SCRIPT -> rocprofv3 counter passes over one probe script
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=$1; script=$2
out=gpurun_out/ppmc_$tag; mkdir -p $out
groups=("SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAIT_ANY"
        "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
        "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum")
i=0
for g in "${groups[@]}"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $g --output-format csv -d $out/g$i -o run -- python3 $script > $out/g$i.log 2>&1
  rc=$?; echo "pmc group $i rc=$rc"; [ $rc -gt 1 ] && exit $rc
done
python3 scripts/dump_pmc.py $out | tee $out/summary.txt
