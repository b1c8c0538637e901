"""Summarise tools/runs/pmc_stalls.sh output: mean counter value per launch of the
named kernel, per variant directory.   python tools/pmc_summary.py KERNEL DIR..."""
import csv
import glob
import os
import sys
from collections import defaultdict

kern = sys.argv[1]
for d in sys.argv[2:]:
    vals = defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if kern in r["Kernel_Name"]:
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(d)
    for c, v in sorted(vals.items()):
        print(f"  {c:40s} {sum(v) / len(v):16.1f}")
