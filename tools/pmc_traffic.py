"""Per-launch HBM traffic of the codec kernels from rocprofv3 PMC passes.

  python tools/pmc_traffic.py FETCH_DIR WRITE_DIR OBJECTS OUT.json [K N]

FETCH_DIR / WRITE_DIR hold run_counter_collection.csv of a `--pmc FETCH_SIZE`
and a `--pmc WRITE_SIZE` pass (separate passes: they do not fit one pass on
gfx950) over tools/prof_kernels.py with OBJECTS resident 64 MiB objects.
Both counters are in KiB.  Per MI355X_MICROARCH.md (HBM section) FETCH_SIZE
reports half the bytes of a 16-byte-per-lane streaming read on gfx950, so it
is doubled; WRITE_SIZE is taken as is.  The result is bytes per object, which
bench.py multiplies by its own object count for `roofline.traffic`.  The
trace names carry no template arguments, so each entry records the code shape
(K, N; default 16, 20, the prof_kernels.py workload) and bench.py uses it only
for a run of that shape.
"""
import csv
import json
import sys
from collections import defaultdict


def per_kernel(path, counter):
    acc = defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] == counter:
                acc[r["Kernel_Name"].split("(")[0].split("<")[0].strip()].append(float(r["Counter_Value"]) * 1024)
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main():
    fdir, wdir, objects, out = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4]
    k, n = (int(sys.argv[5]), int(sys.argv[6])) if len(sys.argv) > 6 else (16, 20)
    fetch = per_kernel(f"{fdir}/run_counter_collection.csv", "FETCH_SIZE")
    write = per_kernel(f"{wdir}/run_counter_collection.csv", "WRITE_SIZE")
    res = {}
    for name in sorted(set(fetch) & set(write)):
        if not (name.startswith("k_") or name.startswith("vds_ec_jit_")) or name == "k_fill_splitmix":
            continue
        f2, w = 2 * fetch[name], write[name]
        res[name] = {"bytes_per_object": (f2 + w) / objects, "fetch_bytes_per_object": f2 / objects,
                  "write_bytes_per_object": w / objects, "objects_per_launch": objects, "k": k, "n": n,
                  "source": "rocprofv3 --pmc FETCH_SIZE (x2, gfx950 streaming-read correction) and --pmc "
                            "WRITE_SIZE, separate passes, mean over launches"}
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
