"""Summarise one training step from a rocprofv3 kernel trace: per-kernel time, gaps, span."""
import csv, sys, collections
path = sys.argv[1]
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
if "--all" in sys.argv:   # whole trace (e.g. generation, no optimiser marker)
    seg = rows
elif "--prologue" in sys.argv:   # one step = from the next-to-last prologue launch to the last one
    marks = [i for i, r in enumerate(rows) if "gemm_small_prep" in r["Kernel_Name"]]
    seg = rows[marks[-2]:marks[-1]]
else:
    marks = [i for i, r in enumerate(rows) if "adam" in r["Kernel_Name"] or "tail_kernel" in r["Kernel_Name"]]
    a, b = marks[-2], marks[-1]
    seg = rows[a + 1:b + 1]
t0 = int(seg[0]["Start_Timestamp"]); t1 = int(seg[-1]["End_Timestamp"])
agg = collections.defaultdict(lambda: [0, 0.0])
busy = 0.0; last_end = t0
for r in seg:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    k = r["Kernel_Name"].split("(")[0].replace("void ", "")[:60]
    agg[k][0] += 1; agg[k][1] += (e - s) / 1e3
    busy += max(0, e - max(s, last_end)) / 1e3; last_end = max(last_end, e)
print(f"step span {(t1 - t0) / 1e3:.1f} us, kernels {len(seg)}, union-busy {busy:.1f} us")
for k, (n, us) in sorted(agg.items(), key=lambda x: -x[1][1]):
    print(f"  {k:60s} n={n:4d} total={us:8.1f} us avg={us / n:7.2f}")
if "--overlap" in sys.argv:   # kernels that ran concurrently (e.g. an RCCL kernel beside a sequence kernel)
    iv = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].replace("void ", "")[:50] or "<unnamed>")
          for r in seg]
    for i, (s1, e1, k1) in enumerate(iv):
        for s2, e2, k2 in iv[i + 1:]:
            ov = min(e1, e2) - max(s1, s2)
            if ov > 0:
                print(f"  overlap {ov / 1e3:8.1f} us: {k1} [{(s1 - t0) / 1e3:.1f}, {(e1 - t0) / 1e3:.1f}] "
                      f"| {k2} [{(s2 - t0) / 1e3:.1f}, {(e2 - t0) / 1e3:.1f}]")
if "--timeline" in sys.argv:
    for r in seg:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        print(f"  {(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f}  {r['Kernel_Name'].split('(')[0][:70] or '<unnamed>'}")
