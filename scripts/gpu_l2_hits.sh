#!/bin/bash
# L2 (TCC) hit rate per kernel of the h2048 step: usage gpu_l2_hits.sh [bench args...]
# One counter group, --pmc with --kernel-trace only.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
out=gpurun_out/pmc_l2; mkdir -p $out
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum --output-format csv -d $out -o run -- python3 bench.py --preset h2048 --per-gpu-batch 512 --steps 1 --warmup 1 "$@" > $out/run.log 2>&1
rc=$?; echo "pmc rc=$rc"; [ $rc -ne 0 ] && exit $rc
python3 - "$out" <<'EOF' | tee $out/summary.txt
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.Counter()
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"][:60]
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    if r["Counter_Name"] == "TCC_HIT_sum":
        n[k] += 1
print(f"{'kernel':60s} {'n':>5s} {'hit%':>6s} {'reqM':>8s} {'hbmRdM':>8s}")
for k, c in sorted(acc.items(), key=lambda kv: -(kv[1]["TCC_HIT_sum"] + kv[1]["TCC_MISS_sum"])):
    h, m = c["TCC_HIT_sum"], c["TCC_MISS_sum"]
    print(f"{k:60s} {n[k]:5d} {100 * h / max(1, h + m):6.1f} {(h + m) / 1e6:8.2f} {c['TCC_EA0_RDREQ_sum'] / 1e6:8.2f}")
EOF
