"""Per-dispatch counter medians of one kernel from rocprofv3 --pmc CSV passes.
usage: python tools/sqsum.py KERNEL_SUBSTRING DIR [DIR...]"""
import csv
import glob
import os
import sys
from collections import defaultdict

import numpy as np

pat, dirs = sys.argv[1], sys.argv[2:]
vals = defaultdict(list)
for d in dirs:
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        per = defaultdict(lambda: defaultdict(float))
        for r in csv.DictReader(open(f)):
            if pat not in r["Kernel_Name"]:
                continue
            per[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
        for c, dd in per.items():
            vals[c].extend(dd.values())
for c in sorted(vals):
    print(f"{c} = {np.median(vals[c]):.0f}  (n={len(vals[c])})")
