#!/bin/bash
# Same-box A/B of several builds: "new" = the tree as sent; every other name X = a copy of the tree
# whose extension is replaced by X/_C*.so.  Alternating runs of bench.py.
# usage: gpu_multi_ab.sh "new ab_r3 ..." ROUNDS OUTFILE [bench args]
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
names=$1; rounds=$2; out=$3; shift 3
: > $out
for v in $names; do
  [ $v = new ] && continue
  d=/tmp/gk_ab_$v; rm -rf $d; mkdir -p $d
  tar --exclude=./gpurun_out --exclude=./.git -cf - . | tar -xf - -C $d
  cp $v/_C*.so $d/gru_mpi_cuda_amd/
done
for i in $(seq $rounds); do
  for v in $names; do
    d=$PWD; [ $v != new ] && d=/tmp/gk_ab_$v
    line=$(cd $d && timeout -k 10 300 python bench.py "$@" 2>/dev/null | grep '^{') || { echo "run failed ($v)"; exit 1; }
    echo "{\"build\": \"$v\", \"round\": $i, \"bench\": $line}" >> $out
    echo "$v $i $(echo $line | python3 -c 'import json,sys; print(json.load(sys.stdin)["ms_per_step"])')"
  done
done
