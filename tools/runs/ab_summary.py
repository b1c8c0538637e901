"""Mean / min / max per library of ab_k32.sh's lines (name enc_ms x rep_ms y aot_ms z value v)."""
import collections
import sys

vals = collections.defaultdict(lambda: collections.defaultdict(list))
for line in open(sys.argv[1]):
    f = line.split()
    if len(f) == 9 and f[1] == "enc_ms":
        for key, x in zip(f[1::2], f[2::2]):
            if x != "None":
                vals[f[0]][key].append(float(x))
for name, d in vals.items():
    print(name, "  ".join(f"{k} {sum(v) / len(v):.3f} [{min(v):.3f}, {max(v):.3f}] n={len(v)}" for k, v in d.items()))
