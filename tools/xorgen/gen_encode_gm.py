#!/usr/bin/env python3
"""gen_encode_gm.py -- offline generator of the compile-time XOR programs of the
additive-FFT encode path of k_encode_bs<K,N> (ec_encode.hip).

Replica r of an object holds, stripe by stripe, the stripe polynomial
P(z) = sum_j c_j z^j (c_j = the stripe's K cells, deg P < K) evaluated at
z = r (chunk.h:245-281; points r = 0..N-1 of GF(2^16), poly 0x1100B).  The
points 0..2^m-1 are the F2-span of 1, x, ..., x^(m-1), so all replicas of a
stripe are one additive FFT (Gao & Mateer, "Additive Fast Fourier Transforms
over Finite Fields", 2010): split P on z^2 + z (a Taylor expansion: XORs
only), evaluate the halves on the image subspace after a twist (one constant
multiplication per coefficient), and recombine with one multiplication per
pair of points.  O(N log N) constant multiplications instead of Horner's N K.

The kernel runs it in two phases per 2048-stripe tile (the cells are bit
planes in LDS, one set of 32 stripes per lane):
  1. wave w computes leaves [w K/WV, (w+1) K/WV) of the decomposition (the
     constants at the bottom of the recursion) from the tile's K cells;
     after a barrier the leaves replace the cells in LDS;
  2. wave w evaluates its replicas from the K leaves (the butterflies).
Every constant multiplication becomes a 16x16 bit-matrix; its rows share
XOR pairs by Paar's greedy CSE, and XOR sums fold into 3-input v_bitop3_b32.
The emitted program is simulated here on random bit planes against direct
GF(2^16) evaluation before it is printed.

  python3 tools/xorgen/gen_encode_gm.py K N WAVES > encode_gm_K_N_wW.inc

Status: a measured study, not in the kernel.  Wired into k_encode_bs (round
2), the programs came to 2.3K / 4.0K / 4.5K VALU per wave and tile for
k/n = 16/20, 32/40, 32/64 against Horner's ~2.6K / ~5.6K / ~10K, but the
phase-2 programs need more than 256 VGPRs beside the prefetched tile
(150-480 spilled) and add two barriers per tile.  Same-box A/B, GiB/s of
object bytes: k=16/n=20 1588 vs Horner 1869; k=32/n=40 859 vs 1330; live
k=32/n=64 600-717 vs 636-649.  Kept for the next attempt (a register-
bounded phase 2, e.g. replicas in two LDS-reloading passes).
"""
import functools
import itertools
import random
import sys

POLY = 0x1100B


def gmul(a, b):
    r = 0
    while b:
        if b & 1:
            r ^= a
        b >>= 1
        a <<= 1
        if a & 0x10000:
            a ^= POLY
    return r


def gpow(a, e):
    r = 1
    for _ in range(e):
        r = gmul(r, a)
    return r


def ginv(a):
    return gpow(a, 65534)


def rows_of(c):
    """Bit-matrix of x -> c x: output plane i = XOR of input planes rows[i]."""
    rows = [[] for _ in range(16)]
    for j in range(16):
        v = gmul(c, 1 << j)
        for i in range(16):
            if v >> i & 1:
                rows[i].append(j)
    return rows


def paar(rows):
    """Paar's greedy CSE over XOR rows of atoms: returns (pairs, rows') where
    pairs[t] = (a, b) defines temp ('t', t) and rows' use atoms and temps."""
    rows = [set(r) for r in rows]
    pairs = []
    while True:
        cnt = {}
        for r in rows:
            for a, b in itertools.combinations(sorted(r, key=repr), 2):
                cnt[(a, b)] = cnt.get((a, b), 0) + 1
        if not cnt:
            break
        (a, b), c = max(sorted(cnt.items(), key=lambda kv: repr(kv[0])), key=lambda kv: kv[1])
        if c < 2:
            break
        t = ("t", len(pairs))
        pairs.append((a, b))
        for r in rows:
            if a in r and b in r:
                r.discard(a)
                r.discard(b)
                r.add(t)
    return pairs, rows


@functools.lru_cache(None)
def mul_cost(c):
    if c in (0, 1):
        return 0
    pairs, rows = paar(rows_of(c))
    return len(pairs) + sum(max(0, len(r) - 1) for r in rows)


# ---------------------------------------------------------------- cell DAG
# nodes: ('in', i) | ('x', a, b) | ('m', a, c); None is the zero cell
def xor(a, b):
    if a is None:
        return b
    if b is None:
        return a
    if a == b:
        return None
    a, b = sorted((a, b), key=repr)
    return ("x", a, b)


def mul(a, c):
    if a is None or c == 0:
        return None
    if c == 1:
        return a
    return ("m", a, c)


def taylor(g):
    """g(x) = sum_i (h_i0 + h_i1 x) (x^2 + x)^i: the pairs (h_i0, h_i1)."""
    n = len(g)
    if n <= 2:
        return [tuple(list(g) + [None] * (2 - n))]
    t = 1
    while 4 * t < n:
        t *= 2
    g = list(g) + [None] * (4 * t - n)
    c0, c1, c2, c3 = g[:t], g[t:2 * t], g[2 * t:3 * t], g[3 * t:]
    s23 = [xor(a, b) for a, b in zip(c2, c3)]
    return taylor(c0 + [xor(a, b) for a, b in zip(c1, s23)]) + taylor(s23 + c3)


def span(basis):
    out = []
    for j in range(1 << len(basis)):
        v = 0
        for i, b in enumerate(basis):
            if j >> i & 1:
                v ^= b
        out.append(v)
    return out


def gm(f, basis, leaves):
    """Evaluations of sum_i f_i z^i at span(basis) (index bit i <-> basis[i]);
    the recursion's constants are appended to `leaves`."""
    m = len(basis)
    f = list(f)
    while f and f[-1] is None:
        f.pop()
    if not f:
        return [None] * (1 << m)
    if len(f) == 1:
        leaves.append(f[0])
        return [f[0]] * (1 << m)
    assert m >= 1 and len(f) <= (1 << m)
    if m == 1:
        leaves.extend(f)
        return [f[0], xor(f[0], mul(f[1], basis[0]))]
    # split on the basis element whose powers are cheapest to twist by (1: free)
    best = None
    for p in range(m):
        cost = 0 if basis[p] == 1 else sum(mul_cost(gpow(basis[p], i)) for i in range(1, len(f)) if f[i] is not None)
        if best is None or cost < best[0]:
            best = (cost, p)
    p = best[1]
    order = [i for i in range(m) if i != p] + [p]
    b2 = [basis[i] for i in order]
    bm = b2[-1]
    h = taylor([mul(c, gpow(bm, i)) for i, c in enumerate(f)])
    ibm = ginv(bm)
    gam = [gmul(b, ibm) for b in b2[:-1]]
    dl = [gmul(x, x) ^ x for x in gam]
    u = gm([x[0] for x in h], dl, leaves)
    v = gm([x[1] for x in h], dl, leaves)
    G = span(gam)
    half = 1 << (m - 1)
    out2 = [None] * (1 << m)
    for j in range(half):
        w0 = xor(u[j], mul(v[j], G[j]))
        out2[j] = w0
        out2[j + half] = xor(w0, v[j])
    out = [None] * (1 << m)
    for idx in range(1 << m):
        idx2 = 0
        for pos, i in enumerate(order):
            if idx >> i & 1:
                idx2 |= 1 << pos
        out[idx] = out2[idx2]
    return out


def dag_nodes(roots, stop):
    """Nodes reachable from roots, not descending into `stop`, post-order."""
    seen, order = set(), []

    def walk(e):
        if e is None or e in seen:
            return
        seen.add(e)
        if e in stop or e[0] == "in":
            return
        walk(e[1])
        if e[0] == "x":
            walk(e[2])
        order.append(e)

    for r in roots:
        walk(r)
    return order, seen


def cost(roots, stop):
    nodes, _ = dag_nodes(roots, stop)
    return sum(16 if e[0] == "x" else mul_cost(e[2]) for e in nodes)


# ---------------------------------------------------------------- emission
class Emitter:
    """Plane-level SSA with lazy XOR sums.  A plane is a frozenset of atoms
    (input planes, temps); sums are folded into xor3s only when a value is
    used twice, multiplied, or leaves the function."""

    def __init__(self, uses):
        self.lines = []
        self.ops = []  # (name, [operands]) for the simulation
        self.n = 0
        self.uses = uses
        self.val = {}
        self.loaded = {}

    def tmp(self, operands):
        name = f"v{self.n}"
        self.n += 1
        if len(operands) == 2:
            self.lines.append(f"    const uint32_t {name} = {operands[0]} ^ {operands[1]};")
        else:
            self.lines.append(f"    const uint32_t {name} = xor3({operands[0]}, {operands[1]}, {operands[2]});")
        self.ops.append((name, list(operands)))
        return name

    def fold(self, s):
        """Materialise an XOR sum of atoms as one SSA value."""
        terms = sorted(s)
        if not terms:
            return "0u"
        acc = terms[0]
        rest = terms[1:]
        while rest:
            if len(rest) >= 2:
                acc = self.tmp([acc, rest[0], rest[1]])
                rest = rest[2:]
            else:
                acc = self.tmp([acc, rest[0]])
                rest = []
        return acc

    def materialise(self, e):
        planes = self.val[e]
        if all(len(p) <= 1 for p in planes):
            return planes
        planes = [frozenset([self.fold(p)]) if len(p) > 1 else p for p in planes]
        self.val[e] = planes
        return planes

    def node(self, e):
        if e[0] == "x":
            a, b = self.val[e[1]], self.val[e[2]]
            planes = [pa ^ pb for pa, pb in zip(a, b)]
        else:  # constant multiple: operand planes as single atoms, Paar over the rows
            src = self.materialise(e[1])
            atoms = [next(iter(p)) if p else None for p in src]
            rows = [[atoms[j] for j in r if atoms[j] is not None] for r in rows_of(e[2])]
            pairs, rows2 = paar(rows)
            names = {}
            for t, (a, b) in enumerate(pairs):
                names[("t", t)] = self.tmp([names.get(a, a), names.get(b, b)])
            planes = [frozenset(names.get(x, x) for x in r) for r in rows2]
        self.val[e] = planes
        if self.uses.get(e, 0) > 1:
            self.materialise(e)

    def out(self, e):
        if e is None:
            return ["0u"] * 16
        return [next(iter(p)) if p else "0u" for p in self.materialise(e)]


def leaf_rows(leaves, K):
    """Coefficients of each leaf over the K input cells (the decomposition is
    linear: leaf = sum_j M[j] c_j, a sparse row)."""
    @functools.lru_cache(None)
    def coef(e):
        if e is None:
            return (0,) * K
        if e[0] == "in":
            v = [0] * K
            v[e[1]] = 1
            return tuple(v)
        if e[0] == "x":
            return tuple(x ^ y for x, y in zip(coef(e[1]), coef(e[2])))
        return tuple(gmul(x, e[2]) for x in coef(e[1]))

    return [coef(e) for e in leaves]


def direct_cost(row):
    return sum(mul_cost(c) + 16 for c in row if c)


def emit_direct(rows, slots):
    """Phase 1 as sparse multiply-accumulate: stream over the input cells, for
    each one add c * cell into the accumulators of the leaves it feeds (the
    constants' bit-matrices for one cell share Paar pairs).  Few live values:
    the accumulators, one cell and its temps."""
    em = Emitter({})
    K = len(rows[0]) if rows else 0
    acc = [[frozenset() for _ in range(16)] for _ in rows]
    for j in range(K):
        feeds = [(i, r[j]) for i, r in enumerate(rows) if r[j]]
        if not feeds:
            continue
        nm = f"c{j}"
        em.lines.append("    __builtin_amdgcn_sched_barrier(0);")
        em.lines.append(f"    const Plane16 {nm} = ld(IC<{j}>{{}});")
        em.loaded[nm] = j
        atoms = [f"{nm}.p[{b}]" for b in range(16)]
        allrows = []
        for i, c in feeds:
            allrows += [[atoms[x] for x in r] for r in rows_of(c)]
        pairs, rows2 = paar(allrows)
        names = {}
        for t, (a, b) in enumerate(pairs):
            names[("t", t)] = em.tmp([names.get(a, a), names.get(b, b)])
        for q, (i, c) in enumerate(feeds):
            for b in range(16):
                terms = acc[i][b] ^ frozenset(names.get(x, x) for x in rows2[16 * q + b])
                if len(terms) > 2:
                    terms = frozenset([em.fold(terms)])
                acc[i][b] = terms
    outs = []
    for i in range(len(rows)):
        outs.append([em.fold(p) if len(p) > 1 else (next(iter(p)) if p else "0u") for p in acc[i]])
    return em, outs


def build(K, N, WV):
    m = (N - 1).bit_length()
    basis = [1 << i for i in range(m)]
    f = [("in", i) for i in range(K)]
    leaves = []
    out = gm(f, basis, leaves)
    pts = span(basis)
    # the DAG against Horner on random cells
    rng = random.Random(K * 1000 + N)
    inp = [rng.randrange(65536) for _ in range(K)]

    @functools.lru_cache(None)
    def ev(e):
        if e is None:
            return 0
        if e[0] == "in":
            return inp[e[1]]
        if e[0] == "x":
            return ev(e[1]) ^ ev(e[2])
        return gmul(ev(e[1]), e[2])

    for idx, pt in enumerate(pts):
        ref = 0
        for j in reversed(range(K)):
            ref = gmul(ref, pt) ^ inp[j]
        assert ev(out[idx]) == ref, (idx, pt)
    leaves = list(dict.fromkeys(x for x in leaves if x is not None))
    assert len(leaves) <= K
    leaves += [None] * (K - len(leaves))
    per = K // WV
    # leaves to waves (per each) by decreasing direct cost, least-loaded first
    rows = leaf_rows(leaves, K)
    load = [0] * WV
    slots = [[] for _ in range(WV)]
    for i in sorted(range(K), key=lambda i: (-direct_cost(rows[i]), i)):
        w = min((w for w in range(WV) if len(slots[w]) < per), key=lambda w: (load[w], w))
        slots[w].append(i)
        load[w] += direct_cost(rows[i])
    order = [i for w in range(WV) for i in sorted(slots[w])]
    leaves = [leaves[i] for i in order]
    lslot = {e: i for i, e in enumerate(leaves) if e is not None}
    lstop = set(lslot)
    rep_node = {r: out[pts.index(r)] for r in range(N)}
    # phase-2 assignment: waves in turn take the costliest free replica, then
    # the replicas sharing most of its butterflies (least marginal cost)
    rpw = (N + WV - 1) // WV
    rows = leaf_rows(leaves, K)
    free = set(range(N))
    reps = [[] for _ in range(WV)]
    quota = [N // WV + (1 if w < N % WV else 0) for w in range(WV)]
    for w in range(WV):
        while len(reps[w]) < quota[w]:
            base = cost([rep_node[x] for x in reps[w]], lstop)
            r = min(free, key=lambda r: (cost([rep_node[x] for x in reps[w] + [r]], lstop) - base
                                         if reps[w] else -cost([rep_node[r]], lstop), r))
            reps[w].append(r)
            free.discard(r)
    return leaves, rows, lslot, rep_node, reps, per, rpw


def emit_phase(roots, stop, load_name, load_slot, sink):
    """Program for roots from the atoms of `stop` cells (loaded with load_name)
    -> (lines, ops, outputs)."""
    nodes, _ = dag_nodes(roots, stop)
    uses = {}
    for e in nodes:
        for o in ([e[1], e[2]] if e[0] == "x" else [e[1]]):
            if o is not None:
                uses[o] = uses.get(o, 0) + 1
    for r in roots:
        if r is not None:
            uses[r] = uses.get(r, 0) + 1
    em = Emitter(uses)
    loaded = {}

    def ensure(e):
        if e in em.val or e is None:
            return
        if e in stop or e[0] == "in":
            slot = load_slot(e)
            nm = f"{load_name}{slot}"
            em.lines.append("    __builtin_amdgcn_sched_barrier(0);")
            em.lines.append(f"    const Plane16 {nm} = ld(IC<{slot}>{{}});")
            loaded[nm] = slot
            em.val[e] = [frozenset([f"{nm}.p[{b}]"]) for b in range(16)]
            return
        ensure(e[1])
        if e[0] == "x":
            ensure(e[2])
        em.node(e)

    results = []
    for i, r in enumerate(roots):
        ensure(r)
        planes = em.out(r)
        results.append(planes)
        sink(em, i, planes)
    return em, loaded, results


def simulate(em, loaded, results, inputs):
    """Run the SSA program on 64-bit words: inputs[slot][b] -> output planes."""
    env = {}
    for nm, slot in loaded.items():
        for b in range(16):
            env[f"{nm}.p[{b}]"] = inputs[slot][b]
    env["0u"] = 0
    for name, ops in em.ops:
        v = 0
        for o in ops:
            v ^= env[o]
        env[name] = v
    return [[env[p] for p in planes] for planes in results]


def bitslice(cells):
    """64 lanes of cells -> 16 planes (bit b of lane l = bit b of cells[l])."""
    return [sum(((c >> b) & 1) << l for l, c in enumerate(cells)) for b in range(16)]


def main():
    K, N, WV = (int(x) for x in sys.argv[1:4])
    leaves, rows, lslot, rep_node, reps, per, rpw = build(K, N, WV)
    rng = random.Random(7)
    lanes = 64
    cells = [[rng.randrange(65536) for _ in range(lanes)] for _ in range(K)]  # cells[j][lane]
    in_planes = [bitslice(c) for c in cells]

    @functools.lru_cache(None)
    def ev_lane(e, lane):
        if e is None:
            return 0
        if e[0] == "in":
            return cells[e[1]][lane]
        if e[0] == "x":
            return ev_lane(e[1], lane) ^ ev_lane(e[2], lane)
        return gmul(ev_lane(e[1], lane), e[2])

    leaf_planes = [bitslice([ev_lane(e, l) for l in range(lanes)]) for e in leaves]
    body = []
    total = [0, 0]
    for w in range(WV):
        mine = leaves[w * per:(w + 1) * per]
        lines1 = []

        def sink1(em, i, planes):
            em.lines.append(f"    L[{i}] = Plane16{{{{{', '.join(planes)}}}}};")

        em1, res1 = emit_direct(rows[w * per:(w + 1) * per], None)
        for i, planes in enumerate(res1):
            sink1(em1, i, planes)
        got = simulate(em1, em1.loaded, res1, in_planes)
        for i, e in enumerate(mine):
            assert got[i] == bitslice([ev_lane(e, l) for l in range(lanes)]), ("leaf", w, i)

        def sink2(em, i, planes):
            em.lines.append(f"    st(IC<{i}>{{}}, Plane16{{{{{', '.join(planes)}}}}});")
            em.lines.append("    __builtin_amdgcn_sched_barrier(0);")

        roots = [rep_node[r] for r in reps[w]]
        em2, ld2, res2 = emit_phase(roots, set(lslot), "l", lambda e: lslot[e], sink2)
        got = simulate(em2, ld2, res2, leaf_planes)
        for i, r in enumerate(reps[w]):
            want = []
            for l in range(lanes):
                acc = 0
                for j in reversed(range(K)):
                    acc = gmul(acc, r) ^ cells[j][l]
                want.append(acc)
            assert got[i] == bitslice(want), ("replica", w, r)
        total[0] += len(em1.ops)
        total[1] += len(em2.ops)
        body.append(f"template <>\nstruct EncodeGm<{K}, {N}, {WV}, {w}> {{")
        body.append(f"  static constexpr int kLeaf0 = {w * per};  // leaves kLeaf0 .. kLeaf0 + {per} - 1")
        body.append(f"  static constexpr int kReps = {len(reps[w])};")
        body.append(f"  static constexpr int kRep[{rpw}] = {{{', '.join(str(r) for r in reps[w] + [-1] * (rpw - len(reps[w])))}}};")
        body.append(f"  // {len(em1.ops)} + {len(em2.ops)} VALU")
        body.append("  template <class LD>")
        body.append(f"  VDS_DEV static void leaves(LD &&ld, Plane16 (&L)[{per}]) {{")
        body.extend(em1.lines)
        body.append("  }")
        body.append("  template <class LD, class ST>")
        body.append("  VDS_DEV static void replicas(LD &&ld, ST &&st) {")
        body.extend(em2.lines)
        body.append("  }")
        body.append("};")
    print(f"// GENERATED by tools/xorgen/gen_encode_gm.py {K} {N} {WV} -- do not edit.")
    print(f"// Additive-FFT encode, K = {K}, points 0..{N - 1}, {WV} waves: "
          f"{total[0]} leaf + {total[1]} replica XOR instructions per tile.")
    print(f"template <>\nstruct EncodeGmShape<{K}, {N}, {WV}> {{\n  static constexpr bool kHas = true;\n"
          f"  static constexpr int kLeavesPerWave = {per};\n  static constexpr int kRepsPerWave = {rpw};\n}};")
    print("\n".join(body))


if __name__ == "__main__":
    main()


def max_live(lines):
    """Peak number of live 32-bit values of an emitted program, in program order."""
    import re
    defs, last = {}, {}
    tok = re.compile(r"\b([cl]\d+\.p\[\d+\]|v\d+)\b")
    loads = re.compile(r"const Plane16 ([cl]\d+) = ld")
    for i, ln in enumerate(lines):
        m = loads.search(ln)
        if m:
            for b in range(16):
                defs[f"{m.group(1)}.p[{b}]"] = i
            continue
        m = re.match(r"\s*const uint32_t (v\d+) =", ln)
        if m:
            defs[m.group(1)] = i
        for t in tok.findall(ln):
            if t in defs and (not m or t != m.group(1)):
                last[t] = i
    ev = [0] * (len(lines) + 1)
    for t, d in defs.items():
        ev[d] += 1
        ev[last.get(t, d) + 1] -= 1
    live = peak = 0
    for x in ev:
        live += x
        peak = max(peak, live)
    return peak
