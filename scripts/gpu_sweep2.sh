#!/bin/bash
# phased-tail knobs + the data-parallel structure (1-rank RCCL) with either tail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
out=gpurun_out/sweep2.jsonl; : > $out
run() {
  local tag="$1" args="$2"; shift 2
  line=$(env "$@" timeout -k 10 200 python bench.py --steps 300 --warmup 50 $args 2>/dev/null | grep '^{') || { echo "bench failed ($tag)"; exit 1; }
  echo "{\"tag\": \"$tag\", \"args\": \"$args\", \"env\": \"$*\", \"ms\": $(echo $line | python3 -c 'import json,sys; print(json.load(sys.stdin)["ms_per_step"])')}" >> $out
  tail -1 $out
}
for cfg in "GK_FC_SMALL_K=2048" "GK_FC_SMALL_K=512" "GK_DEFER_MAX_SPLITS=16" "GK_DEFER_SLABS=0" "GK_TAIL_OCC=4"; do
  run default "" GK_NOP=1
  run "$cfg" "" $cfg
done
for i in 1 2 3; do
  run dp_phased "--rccl-self" GK_TAIL=0
  run dp_fused "--rccl-self" GK_TAIL=1
done
