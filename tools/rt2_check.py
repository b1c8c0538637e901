"""RT2 decomposition check (ec_internal.hpp SynBatchRt): for random
first-k-found survivor sets of k = 32 among 64 ids and random (non-codeword) values,
P(e_m) = sum_j c[m][j] (y(b_j) + P0(b_j)) equals Lagrange over the 32 slots.  CPU only.
  python tools/rt2_check.py"""
import random
POLY=0x1100B
def mul(a,b):
    r=0
    while b:
        if b&1: r^=a
        b>>=1; a<<=1
        if a&0x10000: a^=POLY
    return r
def pw(a,e):
    r=1
    while e:
        if e&1: r=mul(r,a)
        a=mul(a,a); e>>=1
    return r
def inv(a): return pw(a,65534)
def lag_eval(pts, vals, x):
    s=0
    for j,(p,v) in enumerate(zip(pts,vals)):
        num=den=1
        for i,q in enumerate(pts):
            if i!=j: num=mul(num,x^q); den=mul(den,p^q)
        s^=mul(v,mul(num,inv(den)))
    return s
random.seed(5)
K=32
for trial in range(3):
    # random survivors: first 32 found among 0..63 with loss
    alive=[i for i in range(64) if random.random()>0.25][:K]
    E=[e for e in range(K) if e not in alive]
    A=[a for a in range(K) if a in alive]
    B=[b for b in alive if b>=K]
    assert len(B)==len(E)
    vals={p:random.randrange(65536) for p in alive}  # arbitrary (non-codeword) values
    truth=[lag_eval(alive,[vals[p] for p in alive],e) for e in E]
    # P0: values on U with zeros at E
    U=list(range(K)); y0=[vals[u] if u in vals and u<K else 0 for u in U]
    # PERM weights l_c(32)
    lw=[]
    for c in U:
        num=den=1
        for u in U:
            if u!=c: num=mul(num,K^u); den=mul(den,c^u)
        lw.append(mul(num,inv(den)))
    def P0(b):
        t=b-K; s=0
        for c in U: s^=mul(lw[c], y0[c^t])
        return s
    r=[vals[b]^P0(b) for b in B]
    def Z(x):
        p=1
        for a in A: p=mul(p,x^a)
        return p
    got=[]
    for m,e in enumerate(E):
        s=0
        for j,b in enumerate(B):
            num=Z(e); den=Z(b)
            for i,bi in enumerate(B):
                if i!=j: num=mul(num,e^bi); den=mul(den,b^bi)
            s^=mul(r[j],mul(num,inv(den)))
        got.append(s)
    print(len(E), got==truth)
