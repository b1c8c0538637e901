"""Per-kernel PMC means of the live-shape run (tools/runs/profile_round6.sh
b5b: rocprofv3 -T truncates kernel names, so the k_restore_syn dispatches are
told apart by their neighbours): RT = the dispatch right after k_rt_coefs,
MULTI = the others; restore / regenerate by whether k_regen_tail_batch
follows the call.  Prints per class the mean counter values per dispatch and
per 2048-stripe tile.
  python tools/pmc_live_split.py DIR [DIR...]"""
import collections
import csv
import os
import sys

rows = []
for d in sys.argv[1:]:
    rows += list(csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))))
disp = {}
for r in rows:
    k = (r["Counter_Name"].startswith("SQ_INSTS_LDS") or True, int(r["Dispatch_Id"]))
    disp.setdefault(int(r["Dispatch_Id"]), {"name": r["Kernel_Name"], "grid": int(r["Grid_Size"]),
                                            "vgpr": int(r["VGPR_Count"]), "c": {}})["c"][r["Counter_Name"]] = float(r["Counter_Value"])
ids = sorted(disp)
cls = {}
for i, d in enumerate(ids):
    if disp[d]["name"] != "k_restore_syn":
        continue
    prev = disp[ids[i - 1]]["name"] if i else ""
    nxt = [disp[x]["name"] for x in ids[i + 1:i + 3]]
    kind = "RT" if prev == "k_rt_coefs" else "MULTI"
    kind += " regenerate" if "k_regen_tail_batch" in nxt else " restore"
    cls.setdefault(kind, []).append(d)
for kind, ds in sorted(cls.items()):
    acc = collections.defaultdict(list)
    for d in ds:
        for c, v in disp[d]["c"].items():
            acc[c].append(v)
    print(f"{kind}: {len(ds)} dispatches, VGPRs {sorted({disp[d]['vgpr'] for d in ds})}")
    for c, v in sorted(acc.items()):
        print(f"  {c:28s} {sum(v) / len(v):16.1f}")
