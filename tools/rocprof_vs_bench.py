"""Reproduce bench.py's per-kernel launch times from a rocprofv3 summary.

bench.py measures each roofline kernel with HIP events around its launches
(`avg_launch_ms` in the `roofline` blocks: the headline's repair and encode,
the AOT restore, C4's encode / survivor-set repair / AOT repair).  The same
command under `rocprofv3 --kernel-trace --stats` lists every kernel symbol's
average duration; the run-time compiled kernels carry their survivor set in
the symbol (vds_ec_jit.cpp kernel_name), so each has a line of its own.
Prints one row per roofline kernel: the bench's ms, rocprof's average ms and
their ratio.

  python tools/rocprof_vs_bench.py BENCH_LOG run_kernel_stats.csv
"""
import csv
import json
import sys


def main() -> int:
    lines = [l for l in open(sys.argv[1]).read().splitlines() if l.startswith('{"metric"')]
    bench = json.loads(lines[-1])  # (rocprofv3 prints after the bench line)
    stats = {}
    for r in csv.DictReader(open(sys.argv[2])):
        stats[r["Name"]] = (float(r["AverageNs"]) * 1e-6, int(r["Calls"]))
    rows = []
    rf = bench["roofline"]
    rows.append(("headline repair", rf["kernels"]["repair"], rf["avg_launch_ms"] if rf["kernel"] == rf["kernels"]["repair"] else bench["repair_ms"]))
    rows.append(("headline encode", rf["kernels"]["encode"], bench["encode_ms"]))
    if bench.get("restore_aot"):
        rows.append(("headline AOT repair", bench["restore_aot"]["kernel"], bench["restore_aot_ms"]))
    c4 = bench.get("c4") or {}
    for leg, r in (c4.get("roofline") or {}).items():
        if r:
            rows.append((f"C4 {leg}", r["kernel"], r["avg_launch_ms"]))

    def find(sym):
        # rocprof prints "void vds_ec::k_restore_syn<16, 20, 4, false, false, false, vds_ec::NoFill>(...)";
        # bench.py names "k_restore_syn<16,20>" (the one-object-set restore) and "k_encode_bs<16,20>"
        if sym in stats:
            return sym
        if "<" not in sym:
            return None
        base, args = sym.split("<")[0], [a.strip() for a in sym.split("<")[1].rstrip(">").split(",")]
        head = f"{base}<{', '.join(args)}, "
        cands = [n for n in stats if head in n]
        if base == "k_restore_syn":
            cands = [n for n in cands if n.split(head)[1].split(",", 1)[1].startswith(" false, false, false, vds_ec::NoFill>")]
        return max(cands, key=lambda n: stats[n][1]) if cands else None

    print(f"{'leg':22s} {'kernel':44s} {'bench ms':>9s} {'rocprof ms':>10s} {'calls':>6s} {'ratio':>6s}")
    for leg, sym, ms in rows:
        name = find(sym)
        if name is None:
            print(f"{leg:22s} {sym:44s} {ms:9.3f} {'(none)':>10s}")
            continue
        avg, calls = stats[name]
        print(f"{leg:22s} {sym:44s} {ms:9.3f} {avg:10.3f} {calls:6d} {avg / ms:6.3f}")
        print(f"{'':22s}   rocprof symbol: {name[:110]}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
