"""Per-kernel mean of every collected counter over its dispatches (rocprofv3 --pmc CSVs)."""
import csv, glob, os, sys
from collections import defaultdict
root = sys.argv[1]
vals = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(root, "g*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name", "?").split("(")[0].replace("void ", "")[:50]
        vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, c in vals.items():
    print(k)
    for n, v in sorted(c.items()):
        print(f"   {n:32s} {sum(v) / len(v):16.1f}")
