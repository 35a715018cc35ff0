#!/bin/bash
# session 13: group staging straight from the batch list (no numpy stack): multi-step graph tests, then
# the driver's 20-step form, new vs old Python path (ab_old/trainer.py), alternating, same box
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread -k "steps or group or graph" > gpurun_out/s13_tests.log 2>&1
rc=$?; tail -3 gpurun_out/s13_tests.log; [ $rc -ne 0 ] && exit $rc
old=/tmp/gk_ab_old; rm -rf $old; mkdir -p $old
tar --exclude=./gpurun_out --exclude=./.git -cf - . | tar -xf - -C $old
cp ab_old/trainer.py $old/gru_mpi_cuda_amd/engine/trainer.py
out=gpurun_out/s13_ab.txt; : > $out
for i in 1 2 3 4; do
  for v in new old; do
    d=$PWD; [ $v = old ] && d=$old
    ms=$(cd $d && timeout -k 10 200 python bench.py --steps 20 --warmup 5 2>/dev/null | grep -o '"ms_per_step": [0-9.]*') || exit 1
    echo "$v $i $ms" | tee -a $out
  done
done
