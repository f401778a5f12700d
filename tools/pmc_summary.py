"""Average per-dispatch counter values per kernel from rocprofv3 --pmc csv directories."""
import collections
import csv
import glob
import os
import sys

acc = collections.defaultdict(lambda: collections.defaultdict(list))
for d in sys.argv[1:]:
    for f in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
        per = collections.defaultdict(float)
        names = {}
        for r in csv.DictReader(open(f)):
            key = (r["Dispatch_Id"], r["Counter_Name"])
            per[key] += float(r["Counter_Value"])
            names[r["Dispatch_Id"]] = r["Kernel_Name"]
        for (disp, cn), v in per.items():
            acc[names[disp][:48]][cn].append(v)
for k, cs in sorted(acc.items()):
    print(k)
    print("   " + "  ".join(f"{cn}={sum(v) / len(v):.4g}" for cn, v in sorted(cs.items())))
