"""Model of bls_w12d.h inv_wave: Bernstein-Yang safegcd (30-divstep batches, variable time)
with the 13 signed 30-bit limbs of d, e, f, g held one per lane, REDUNDANT after each batch
(one carry pass instead of a ripple), sign tests on the top limb only, and the exit test
normalizing g only when its low 30 bits vanish.  Checks the inverse of 3000 random inputs and
prints the batch-count histogram.  Test infrastructure: nothing imports it."""
import random
P = 0x1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaaab
NL, M30 = 13, (1 << 30) - 1
def limbs(x): return [(x >> (30*i)) & M30 for i in range(NL)]
def val(l): return sum(v << (30*i) for i, v in enumerate(l))
def sra(x, n): return x >> n  # python >> is arithmetic
def divsteps30(eta, f, g):
    u, v, q, r = 1, 0, 0, 1; i = 30
    M32 = (1 << 32) - 1
    f &= M32; g &= M32
    while True:
        gi = g | ((M32 << i) & M32)
        zeros = (gi & -gi).bit_length() - 1
        g = (g >> zeros) & M32; u = (u << zeros) & M32; v = (v << zeros) & M32
        eta -= zeros; i -= zeros
        if i == 0: break
        if eta < 0:
            eta = -eta; f, g = g, (-f) & M32; u, q = q, (-u) & M32; v, r = r, (-v) & M32
        limit = min(eta + 1, i)
        m = M32 >> (32 - limit)
        w = ((-g) * pow(f, -1, 1 << 32)) & m
        g = (g + f * w) & M32; q = (q + u * w) & M32; r = (r + v * w) & M32
    s = lambda x: x - (1 << 32) if x >> 31 else x
    return eta, s(u), s(v), s(q), s(r)
def shift_recombine(t):  # t: per-lane int64 sums; returns new redundant limbs of sum t_i 2^(30(i-1))
    lo = [x & M30 for x in t]; hi = [sra(x, 30) for x in t]
    n = [(lo[j+1] if j+1 < NL else 0) + hi[j] for j in range(NL)]
    # one parallel normalization pass (top limb keeps its sign)
    c = [sra(x, 30) for x in n]
    out = [((n[j] & M30) if j < NL-1 else n[j]) + (c[j-1] if j > 0 else 0) for j in range(NL)]
    out[NL-1] = n[NL-1] + c[NL-2]
    return out
def inverse(x):
    Pl = limbs(P); pinv30 = pow(P, -1, 1 << 30)
    f, g, d, e = Pl[:], limbs(x), [0]*NL, [1] + [0]*(NL-1)
    eta = -1; nb = 0
    for b in range(37):
        eta, u, v, q, r = divsteps30(eta, f[0] & M30, g[0] & M30)
        # d, e
        sd = -1 if d[NL-1] < 0 else 0; se = -1 if e[NL-1] < 0 else 0
        md = (u & sd) + (v & se); me = (q & sd) + (r & se)
        cd = (u*d[0] + v*e[0]); ce = (q*d[0] + r*e[0])
        md -= (pinv30*cd + md) & M30; me -= (pinv30*ce + me) & M30
        td = [u*d[i] + v*e[i] + Pl[i]*md for i in range(NL)]
        te = [q*d[i] + r*e[i] + Pl[i]*me for i in range(NL)]
        assert val(td) % (1 << 30) == 0 and val(te) % (1 << 30) == 0
        d, e = shift_recombine(td), shift_recombine(te)
        tf = [u*f[i] + v*g[i] for i in range(NL)]; tg = [q*f[i] + r*g[i] for i in range(NL)]
        f, g = shift_recombine(tf), shift_recombine(tg)
        for a in (d, e, f, g): assert all(-(1 << 5) <= a[j] < (1 << 30) + (1 << 5) for j in range(NL-1)), a
        nb = b + 1
        if (g[0] & M30) == 0 and val(g) == 0: break
    F, D = val(f), val(d)
    assert F in (1, -1), F
    return (D * F) % P, nb
import collections
rng = random.Random(5); mx = 0; hist = collections.Counter()
for t in range(3000):
    x = rng.randrange(1, P) if t > 3 else [1, 2, P-1, P-2][t]
    y, nb = inverse(x); mx = max(mx, nb); hist[nb] += 1
    assert y * x % P == 1
print("ok, max batches", mx, sorted(hist.items()))
