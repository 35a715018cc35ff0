#!/bin/bash
# headline knob sweep on the current tree: each setting against an interleaved default run
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
out=gpurun_out/sweep.jsonl; : > $out
run() {
  local tag="$1"; shift
  line=$(env "$@" timeout -k 10 200 python bench.py --steps 300 --warmup 50 2>/dev/null | grep '^{') || { echo "bench failed ($tag)"; exit 1; }
  echo "{\"tag\": \"$tag\", \"env\": \"$*\", \"ms\": $(echo $line | python3 -c 'import json,sys; print(json.load(sys.stdin)["ms_per_step"])')}" >> $out
  tail -1 $out
}
for cfg in "GK_TAIL_OCC=4" "GK_TAIL_FC=0" "GK_TAIL_FC_WAIT=1" "GK_TAIL_ADAM_WAIT=1" "GK_TAIL_BATCH=1" "GK_FWD_RS=1" "GK_FC_SMALL_K=512" "GK_DEFER_MAX_SPLITS=4" "GK_P_SLABS=2" "GK_BWD_DH=1" "GK_TAIL=0"; do
  run default GK_NOP=1
  run "$cfg" $cfg
done
run default GK_NOP=1
