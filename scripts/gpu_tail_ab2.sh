#!/bin/bash
# fused vs phased step tail (and dW_fc placement) on the current tree, alternating, + traces
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
out=gpurun_out/tail_ab2.jsonl; : > $out
run() {
  local tag="$1"; shift
  line=$(env "$@" timeout -k 10 200 python bench.py --steps 300 --warmup 50 2>/dev/null | grep '^{') || { echo "bench failed ($tag)"; exit 1; }
  echo "{\"tag\": \"$tag\", \"ms\": $(echo $line | python3 -c 'import json,sys; print(json.load(sys.stdin)["ms_per_step"])')}" >> $out
  tail -1 $out
}
for i in 1 2 3 4; do
  run fused GK_NOP=1
  run phased GK_TAIL=0
  run fused_fc0 GK_TAIL_FC=0
done
for i in 1 2; do
  line=$(timeout -k 10 200 python bench.py --steps 20 --warmup 5 2>/dev/null | grep "^{") && echo "{\"tag\": \"driver_fused\", \"ms\": $(echo $line | python3 -c "import json,sys; print(json.load(sys.stdin)[\"ms_per_step\"])")}" >> $out && tail -1 $out
  line=$(GK_TAIL=0 timeout -k 10 200 python bench.py --steps 20 --warmup 5 2>/dev/null | grep "^{") && echo "{\"tag\": \"driver_phased\", \"ms\": $(echo $line | python3 -c "import json,sys; print(json.load(sys.stdin)[\"ms_per_step\"])")}" >> $out && tail -1 $out
done
GK_TAIL=0 bash scripts/gpu_prof.sh phased --steps 20 --warmup 4 | head -12
