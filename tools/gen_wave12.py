#!/usr/bin/env python3
"""Generate grandine_amd/csrc/bls_wave12_tables.h: the linear maps of the wave-
cooperative Fp12 product (bls_wave12.h).

An Fp12 product c = a*b is computed by one wavefront as
  PRE   lane l < 54: L_l = sum of <= 8 coefficients of a, R_l = same of b
  MUL   lane l < 54: p_l = L_l * R_l          (one Montgomery product per lane)
  POST1 lane l < 36: Fp2 Karatsuba recombination   (<= 3 signed terms)
  POST2 lane l < 18: Fp6 Karatsuba recombination   (<= 6 signed terms, xi folded in)
  POST3 lane l < 12: Fp12 Karatsuba recombination  (<= 4 signed terms, v folded in)
i.e. three-level Karatsuba (Fp12 over Fp6 over Fp2 over Fp): 54 Fp products, one per
lane, in a single round.  Coefficient index of an Fp12 value (bls_field.h tower):
    idx = h*6 + j*2 + k   for  c_h (w-part) . c_j (v-part) . c_k (u-part).
The value space of the POST rounds is [p_0..p_53 | POST1 outputs | POST2 outputs].

Run:  python tools/gen_wave12.py > grandine_amd/csrc/bls_wave12_tables.h
"""


def idx(h, j, k):
    return h * 6 + j * 2 + k


def build():
    """(prod, post1, post2, post3): the 54 product operand sets and the three recombination
    rounds as (value index, sign) lists (value space [p_0..p_53 | POST1 | POST2])."""
    # ---- products: (i6, j, k) with i6 in {0: a0*b0, 1: a1*b1, 2: (a0+a1)(b0+b1)},
    # j the Fp6 Karatsuba product, k the Fp2 Karatsuba product.
    fp6_sets = {0: [0], 1: [1], 2: [0, 1]}                 # w-parts summed
    fp2_sets = {0: [0], 1: [1], 2: [2], 3: [1, 2], 4: [0, 1], 5: [0, 2]}  # v-parts
    fp_sets = {0: [0], 1: [1], 2: [0, 1]}                  # u-parts
    prod = []  # list of (subset of coef indices)
    pid = {}
    for i6 in range(3):
        for j in range(6):
            for k in range(3):
                s = sorted(idx(h, jj, kk) for h in fp6_sets[i6] for jj in fp2_sets[j] for kk in fp_sets[k])
                pid[(i6, j, k)] = len(prod)
                prod.append(s)
    assert len(prod) == 54 and max(len(s) for s in prod) == 8

    # ---- POST1: Fp2 recombination of each (i6, j): e0 = p0 - p1, e1 = p2 - p0 - p1
    post1 = []
    v1 = {}
    base1 = 54
    for i6 in range(3):
        for j in range(6):
            p0, p1, p2 = (pid[(i6, j, k)] for k in range(3))
            v1[(i6, j, 0)] = base1 + len(post1)
            post1.append([(p0, 1), (p1, -1)])
            v1[(i6, j, 1)] = base1 + len(post1)
            post1.append([(p2, 1), (p0, -1), (p1, -1)])
    assert len(post1) == 36

    # ---- POST2: Fp6 recombination for each i6, over Fp2 values given as (c0 terms, c1 terms)
    def f2(i6, j):
        return ({v1[(i6, j, 0)]: 1}, {v1[(i6, j, 1)]: 1})

    def add(x, y, s=1):
        r = dict(x)
        for kk, vv in y.items():
            r[kk] = r.get(kk, 0) + s * vv
            if r[kk] == 0:
                del r[kk]
        return r

    def f2add(x, y, s=1):
        return (add(x[0], y[0], s), add(x[1], y[1], s))

    def f2xi(x):  # (x0 + x1 u)(1 + u) = (x0 - x1) + (x0 + x1) u
        return (add(x[0], x[1], -1), add(x[0], x[1], 1))

    post2 = []
    v2 = {}
    base2 = base1 + 36
    for i6 in range(3):
        T0, T1, T2, M12, M01, M02 = (f2(i6, j) for j in range(6))
        c0 = f2add(T0, f2xi(f2add(f2add(M12, T1, -1), T2, -1)))
        c1 = f2add(f2add(f2add(M01, T0, -1), T1, -1), f2xi(T2))
        c2 = f2add(f2add(f2add(M02, T0, -1), T2, -1), T1)
        for jj, c in enumerate((c0, c1, c2)):
            for kk in range(2):
                v2[(i6, jj, kk)] = base2 + len(post2)
                post2.append(sorted(c[kk].items()))
    assert len(post2) == 18

    # ---- POST3: C1 = S - T0 - T1, C0 = T0 + v*T1 with v*(x0,x1,x2) = (xi x2, x0, x1)
    post3 = [None] * 12
    for jj in range(3):
        for kk in range(2):
            post3[idx(1, jj, kk)] = [(v2[(2, jj, kk)], 1), (v2[(0, jj, kk)], -1), (v2[(1, jj, kk)], -1)]
    # C0_j = T0_j + (v T1)_j
    for jj in range(3):
        for kk in range(2):
            terms = {v2[(0, jj, kk)]: 1}
            if jj == 0:  # xi * T1_2
                x0, x1 = v2[(1, 2, 0)], v2[(1, 2, 1)]
                if kk == 0:
                    terms = add(terms, {x0: 1, x1: -1})
                else:
                    terms = add(terms, {x0: 1, x1: 1})
            else:
                terms = add(terms, {v2[(1, jj - 1, kk)]: 1})
            post3[idx(0, jj, kk)] = sorted(terms.items())

    for rnd in (post1, post2, post3):
        for terms in rnd:
            assert all(abs(s) == 1 for _, s in terms)
    return prod, post1, post2, post3


def build_sqr():
    """The squaring plan: the same three-level Karatsuba tree applied to a*a, where every leaf
    is an Fp2 SQUARING (x0 + x1)(x0 - x1), x0 x1 -- 36 Fp products instead of 54.  Returns
    (lhs, rhs_pos, rhs_neg, post1, post2, post3): product l is (sum of lhs[l]) * (sum of
    rhs_pos[l] - sum of rhs_neg[l]); the POST rounds as in build(), over [p_0..p_35 | POST1 |
    POST2] (POST1 outputs: c0 = p0, c1 = 2 p1)."""
    fp6_sets = {0: [0], 1: [1], 2: [0, 1]}
    fp2_sets = {0: [0], 1: [1], 2: [2], 3: [1, 2], 4: [0, 1], 5: [0, 2]}
    lhs, rp, rn = [], [], []
    pid = {}
    for i6 in range(3):
        for j in range(6):
            s0 = sorted(idx(h, jj, 0) for h in fp6_sets[i6] for jj in fp2_sets[j])
            s1 = sorted(idx(h, jj, 1) for h in fp6_sets[i6] for jj in fp2_sets[j])
            pid[(i6, j, 0)] = len(lhs)  # (x0 + x1)(x0 - x1)
            lhs.append(sorted(s0 + s1))
            rp.append(s0)
            rn.append(s1)
            pid[(i6, j, 1)] = len(lhs)  # x0 x1
            lhs.append(s0)
            rp.append(s1)
            rn.append([])
    assert len(lhs) == 36 and max(len(x) for x in lhs) == 8 and max(len(x) for x in rp + rn) == 4
    post1 = []
    v1 = {}
    base1 = 36
    for i6 in range(3):
        for j in range(6):
            v1[(i6, j, 0)] = base1 + len(post1)
            post1.append([(pid[(i6, j, 0)], 1)])
            v1[(i6, j, 1)] = base1 + len(post1)
            post1.append([(pid[(i6, j, 1)], 1), (pid[(i6, j, 1)], 1)])
    # POST2 / POST3: build()'s, with the POST1 value indices of this plan
    _, p1ref, p2ref, p3ref = build()
    remap = {}
    for i6 in range(3):
        for j in range(6):
            for k in range(2):
                remap[54 + 2 * (6 * i6 + j) + k] = v1[(i6, j, k)]
    base2 = base1 + 36
    post2 = [[(remap[src], g) for src, g in t] for t in p2ref]
    post3 = [[(base2 + (src - 90), g) for src, g in t] for t in p3ref]
    return lhs, rp, rn, post1, post2, post3


def main():
    prod, post1, post2, post3 = build()
    base1, base2 = 54, 90

    # ---- per-lane plan: the same maps as register-resident byte lists.  Positive terms
    # first, then negative ones, padded to the round's maxima with the zero slot, so that
    # every lane runs the same instruction stream (no sign selects, no divergence).
    zero = base2 + 18          # index of the all-zero value slot in ws
    pre_none = 12              # PRE: "no coefficient" -> zero operand
    rounds = {}
    for name, rnd in (("POST1", post1), ("POST2", post2), ("POST3", post3)):
        npos = max(sum(1 for _, g in t if g > 0) for t in rnd)
        nneg = max(sum(1 for _, g in t if g < 0) for t in rnd)
        assert npos + nneg <= 8          # (npos + nneg) p < 2^384 and 2 plan words
        lanes = []
        for l in range(64):
            t = rnd[l] if l < len(rnd) else []
            pos = [s for s, g in t if g > 0] + [zero] * (npos - sum(1 for _, g in t if g > 0))
            neg = [s for s, g in t if g < 0] + [zero] * (nneg - sum(1 for _, g in t if g < 0))
            lanes.append(pos + neg + [zero] * (8 - npos - nneg))
        rounds[name] = (npos, nneg, lanes)

    def pack(bs):
        return [sum(b << (8 * i) for i, b in enumerate(bs[k:k + 4])) for k in (0, 4)]

    plan = []
    for l in range(64):
        pre = prod[l] + [pre_none] * (8 - len(prod[l])) if l < 54 else [pre_none] * 8
        words = pack(pre)
        for name in ("POST1", "POST2", "POST3"):
            words += pack(rounds[name][2][l])
        plan.append(words)

    out = []
    w = out.append
    w("// GENERATED by tools/gen_wave12.py -- do not edit.")
    w("// Linear maps of the wave-cooperative Fp12 product (three-level Karatsuba, 54 Fp")
    w("// products).  PRE: coefficient indices (-1 = none).  POSTn: (value index, sign).")
    w("#pragma once")
    w("#ifndef GBLS_CONSTANT")
    w("#if defined(__HIP__)")
    w("#define GBLS_CONSTANT __constant__")
    w("#else")
    w("#define GBLS_CONSTANT static const")
    w("#endif")
    w("#endif")
    w("namespace gbls { namespace w12 {")
    w("constexpr int NPROD = 54, NPOST1 = 36, NPOST2 = 18, NPOST3 = 12;")
    w("constexpr int BASE1 = %d, BASE2 = %d, NVAL = %d;" % (base1, base2, base2 + 18))
    w("constexpr int PRE_T = 8, POST1_T = %d, POST2_T = %d, POST3_T = %d;" % (
        max(len(t) for t in post1), max(len(t) for t in post2), max(len(t) for t in post3)))
    w("GBLS_CONSTANT int8_t PRE[54][8] = {")
    for s in prod:
        w("  {%s}," % ", ".join(str(x) for x in (s + [-1] * (8 - len(s)))))
    w("};")
    for name, rnd in (("POST1", post1), ("POST2", post2), ("POST3", post3)):
        T = max(len(t) for t in rnd)
        w("// (src, sign) pairs; src -1 = none")
        w("GBLS_CONSTANT int16_t %s[%d][%d][2] = {" % (name, len(rnd), T))
        for terms in rnd:
            cells = ["{%d, %d}" % (s, g) for s, g in terms] + ["{-1, 0}"] * (T - len(terms))
            w("  {%s}," % ", ".join(cells))
        w("};")
    w("// Register plan per lane: words 0-1 PRE bytes, 2-3 POST1, 4-5 POST2, 6-7 POST3;")
    w("// POST bytes: NPOSn positive sources, then NNEGn negative, then padding.")
    w("constexpr int ZERO_SLOT = %d, PRE_NONE = %d, NSLOT = %d;" % (zero, pre_none, zero + 1))
    for i, name in enumerate(("POST1", "POST2", "POST3")):
        w("constexpr int NPOS%d = %d, NNEG%d = %d;" % (i + 1, rounds[name][0], i + 1, rounds[name][1]))
    w("GBLS_CONSTANT uint32_t PLAN[64][8] = {")
    for words in plan:
        w("  {%s}," % ", ".join("0x%08xu" % x for x in words))
    w("};")
    w("}}  // namespace gbls::w12")
    print("\n".join(out))


if __name__ == "__main__":
    main()
