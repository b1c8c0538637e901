"""Mean per dispatch of every PMC counter, per kernel, from rocprofv3
`--pmc ... -f csv` output directories (the *counter_collection.csv files).

  python tools/pmc_kernels.py OUT.json DIR [DIR ...]

Kernels are keyed by name and Kernel_Id: with rocprofv3 -T the names are
truncated, and the instantiations of one template (k_restore_syn's MULTI,
RT, regenerate ...) differ only in the id (match ids to full names with an
untruncated --kernel-trace of the same command).  Also printed as a table."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def short(name):
    name = name.split("(")[0]
    return name.replace("void vds_ec::", "").replace("vds_ec::", "")


def main():
    out, dirs = sys.argv[1], sys.argv[2:]
    acc = defaultdict(lambda: defaultdict(list))
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                key = f'{short(r["Kernel_Name"])} id={r["Kernel_Id"]} vgpr={r["VGPR_Count"]} sgpr={r["SGPR_Count"]}'
                acc[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
    res = {}
    for kn, cs in acc.items():
        res[kn] = {"dispatches": max(len(v) for v in cs.values()),
                   "mean": {c: sum(v) / len(v) for c, v in sorted(cs.items())}}
    json.dump(res, open(out, "w"), indent=1)
    for kn, r in sorted(res.items(), key=lambda x: -x[1]["mean"].get("SQ_WAVES", 0)):
        print(f"{kn[:110]}  n={r['dispatches']}")
        print("   " + "  ".join(f"{c}={v:.4g}" for c, v in r["mean"].items()))


if __name__ == "__main__":
    main()
