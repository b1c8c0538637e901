"""Calibrate the oracle (oracle/vds_oracle.c, the CPU restatement bench.py's
cpu_baseline times) against the survey's timings of the reference's own
chunk_storage.cpp build in this container (k=16,n=20 encode of a
64 MiB object 2.085 s; restore from {4..19} 1.798 s; k=4,n=6 1 MiB encode
12 ms, restore 9 ms; single thread, g++ -O2).  Test infrastructure.

  python tools/calibrate_oracle.py [--reps 3]
"""
import argparse
import json
import os
import platform
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import oracle_ctypes as O  # noqa: E402

SURVEY = {"k16_64MiB_encode_s": 2.085, "k16_64MiB_restore_s": 1.798, "k4_1MiB_encode_s": 0.012,
          "k4_1MiB_restore_s": 0.009}


def best(fn, reps):
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return min(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    O.lib()
    out = {}
    for k, n, size, nodes, tag in ((16, 20, 64 << 20, list(range(4, 20)), "k16_64MiB"),
                                   (4, 6, 1 << 20, [2, 3, 4, 5], "k4_1MiB")):
        d = O.splitmix(0x7664730000000000, size)
        reps = [None] * n
        def enc():
            for r in range(n):
                reps[r] = O.encode(k, r, d)
        out[f"{tag}_encode_s"] = best(enc, a.reps)
        def res():
            assert O.restore(k, nodes, [reps[r] for r in nodes]).size == size
        out[f"{tag}_restore_s"] = best(res, a.reps)
    ratio = {key: round(out[key] / SURVEY[key], 3) for key in SURVEY}
    print(json.dumps({"oracle_s": {kk: round(v, 4) for kk, v in out.items()}, "survey_reference_s": SURVEY,
                      "oracle_over_reference": ratio, "cpu": platform.processor() or platform.machine(),
                      "note": "ratio < 1: the restatement is faster than the reference build on the same host"}))


if __name__ == "__main__":
    main()
