"""Per-kernel PMC summary of a tools/pmc_conv.sh run: mean counter value per dispatch, by kernel."""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1]
vals = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(root, "*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("void ", "").split("(")[0]
        vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in vals.items():
    print(k)
    for c in sorted(d):
        v = d[c]
        print(f"   {c:28s} {sum(v) / len(v):16.1f}   (n={len(v)})")
