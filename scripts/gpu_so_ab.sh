#!/bin/bash
# Same-box A/B of two builds: the tree as sent (new) vs a copy whose extension is replaced by
# ab_old/_C*.so (old), alternating runs of the headline bench.  usage: gpu_so_ab.sh [rounds] [bench args]
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
rounds=${1:-2}; shift
old=/tmp/gk_ab_old; rm -rf $old; mkdir -p $old
tar --exclude=./gpurun_out --exclude=./.git -cf - . | tar -xf - -C $old
cp ab_old/_C*.so $old/gru_mpi_cuda_amd/
for i in $(seq $rounds); do
  for v in new old; do
    d=$PWD; [ $v = old ] && d=$old
    (cd $d && timeout -k 10 200 python bench.py --steps 200 --warmup 30 "$@") > gpurun_out/soab_${v}_$i.log 2>&1
    rc=$?; [ $rc -gt 1 ] && { echo "stop rc=$rc"; exit $rc; }
    echo "$v $i $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/soab_${v}_$i.log)"
  done
done
