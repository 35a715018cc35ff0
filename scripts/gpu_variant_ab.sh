#!/bin/bash
# Same-box A/B of step-plan variants (StepLdsVariants fields, bench.py --variant), alternating runs.
# usage: gpu_variant_ab.sh "fwd_fc=0 fwd_fc=1" ROUNDS OUTFILE [bench args]
#   a variant token may join several fields with commas: "fwd_fc=0,bwd_xring=2"; "-" = defaults
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
vars=$1; rounds=$2; out=$3; shift 3
: > $out
for i in $(seq $rounds); do
  for v in $vars; do
    args=()
    if [ "$v" != "-" ]; then for kv in ${v//,/ }; do args+=(--variant "$kv"); done; fi
    line=$(timeout -k 10 300 python bench.py "${args[@]}" "$@" 2>/dev/null | grep '^{') || { echo "run failed ($v)"; exit 1; }
    echo "{\"variant\": \"$v\", \"round\": $i, \"bench\": $line}" >> $out
    echo "$v $i $(echo $line | python3 -c 'import json,sys; print(json.load(sys.stdin)["ms_per_step"])')"
  done
done
