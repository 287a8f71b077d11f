#!/usr/bin/env python3
"""Generate grandine_amd/csrc/bls_dfp_tables.h: constants of the row-distributed Fp layer
(bls_dfp.h).

An element is spread over a 16-lane DPP row: lane j holds limb j of x = sum l_j 2^(28 j),
Montgomery form with R = 2^448 (16 limbs of 28 bits; p needs 14).  Emitted: the limbs of p
and p' = -p^-1 mod 2^448 (wave-uniform operands of the product), per-lane limbs of the
conversion / bias / Frobenius constants, and the row plans of the Fp12 engine (bls_w12d.h).

Run:  python tools/gen_dfp.py > grandine_amd/csrc/bls_dfp_tables.h
"""

import os
import sys

P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
X_ABS = 0xD201000000010000
N, W = 16, 28
M = (1 << W) - 1
R = 1 << (N * W)


def limbs(x, n=N):
    assert 0 <= x < (1 << (W * n)), hex(x)
    return [(x >> (W * j)) & M for j in range(n)]


def rebalanced(x, borrow):
    """x in 16 limbs where each of limbs 0..12 borrows `borrow` units of 2^28 from the next
    limb (limbs in [borrow 2^28 - borrow, (borrow + 1) 2^28)), so that subtracting limbs
    below that never goes negative; limb 13 keeps the top."""
    l = limbs(x)
    for j in range(13):
        l[j] += borrow << W
        l[j + 1] -= borrow
    assert all((borrow << W) - borrow <= v < ((borrow + 1) << W) for v in l[:13]), l
    assert l[13] >= 0 and l[14] == l[15] == 0, l
    assert sum(v << (W * j) for j, v in enumerate(l)) == x
    return l


def w12d_plan():
    """Per-row plan of the row-distributed Fp12 product (bls_w12d.h): the 54 products of
    tools/gen_wave12.py, then the POST1/POST2 rounds composed into one round R1 (18 values,
    <= 6 positive and <= 6 negative product terms each, counted with multiplicity) and POST3 as round R2 (12 values,
    <= 3 positive and <= 2 negative R1 terms).  Slot space of the workspace:
    [0, 54) products, [54, 72) R1 values, 72 the zero slot; PRE index 12 = zero operand."""
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import gen_wave12
    prod, post1, post2, post3 = gen_wave12.build()
    expr = {i: {i: 1} for i in range(54)}

    def comb(terms):
        r = {}
        for src, g in terms:
            for k, v in expr[src].items():
                r[k] = r.get(k, 0) + g * v
        return {k: v for k, v in r.items() if v}
    for l, t in enumerate(post1):
        expr[54 + l] = comb(t)
    r1 = [comb(t) for t in post2]
    ZERO = 72
    plan_pre = [prod[r] + [12] * (8 - len(prod[r])) for r in range(54)]
    plan_r1 = []
    for o in r1:
        # a coefficient of +-2 appears as a repeated slot
        pos = sorted(k for k, v in o.items() if v > 0 for _ in range(v))
        neg = sorted(k for k, v in o.items() if v < 0 for _ in range(-v))
        assert len(pos) <= 6 and len(neg) <= 6
        plan_r1.append(pos + [ZERO] * (6 - len(pos)) + neg + [ZERO] * (6 - len(neg)))
    plan_r2 = []
    for t in post3:  # indices 90.. of gen_wave12's value space are its POST2 outputs
        pos = [54 + (src - 90) for src, g in t if g > 0]
        neg = [54 + (src - 90) for src, g in t if g < 0]
        assert all(90 <= src < 108 for src, _ in t) and len(pos) <= 3 and len(neg) <= 2
        plan_r2.append(pos + [ZERO] * (3 - len(pos)) + neg + [ZERO] * (2 - len(neg)))
    return plan_pre, plan_r1, plan_r2


def w12d_sqr_plan():
    """Per-row plan of the row-distributed Fp12 SQUARING (bls_w12d.h sqr): 36 products
    (sum of lhs) * (bias + sum of rhs_pos - sum of rhs_neg) of tools/gen_wave12.py build_sqr,
    then R1 (18 values, <= 6 + 6 product terms) and R2 (12 values, <= 3 + 2 R1 terms) in the
    multiply plan's slot space: [0, 36) products, [54, 72) R1 values, 72 the zero slot."""
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import gen_wave12
    lhs, rp, rn, post1, post2, post3 = gen_wave12.build_sqr()
    n = len(lhs)
    expr = {i: {i: 1} for i in range(n)}

    def comb(terms):
        r = {}
        for src, g in terms:
            for k, v in expr[src].items():
                r[k] = r.get(k, 0) + g * v
        return {k: v for k, v in r.items() if v}
    for l, t in enumerate(post1):
        expr[n + l] = comb(t)
    r1 = [comb(t) for t in post2]
    ZERO = 72
    plan_l = [x + [12] * (8 - len(x)) for x in lhs]
    plan_rp = [x + [12] * (4 - len(x)) for x in rp]
    plan_rn = [x + [12] * (4 - len(x)) for x in rn]
    plan_r1 = []
    for o in r1:
        pos = sorted(k for k, v in o.items() if v > 0 for _ in range(v))
        neg = sorted(k for k, v in o.items() if v < 0 for _ in range(-v))
        assert len(pos) <= 6 and len(neg) <= 6
        plan_r1.append(pos + [ZERO] * (6 - len(pos)) + neg + [ZERO] * (6 - len(neg)))
    plan_r2 = []
    base2 = 2 * n
    for t in post3:
        pos = [54 + (src - base2) for src, g in t if g > 0]
        neg = [54 + (src - base2) for src, g in t if g < 0]
        assert all(base2 <= src < base2 + 18 for src, _ in t) and len(pos) <= 3 and len(neg) <= 2
        plan_r2.append(pos + [ZERO] * (3 - len(pos)) + neg + [ZERO] * (2 - len(neg)))
    return plan_l, plan_rp, plan_rn, plan_r1, plan_r2


def mont(x):
    return x * R % P


def gs_plan():
    """Granger-Scott cyclotomic squaring on the row engine (bls_w12d.h cyc_sqr), for elements
    of the cyclotomic subgroup (x^(p^6 + 1) = 1).  With Fp12 = Fp4[w]/(w^3 - s), s = w^3, the
    element is g0 + g1 w + g2 w^2, gi = (z_2i..) pairs of Fp2 coefficients, and
    x^2 = (3 g0^2 - 2 conj(g0)) + (3 s g2^2 + 2 conj(g1)) w + (3 g1^2 - 2 conj(g2)) w^2, each
    Fp4 square (a + b s)^2 = (a^2 + xi b^2) + ((a + b)^2 - a^2 - b^2) s from three Fp2 squares
    (x0 + x1)(x0 - x1), x0 x1.  The -2 z / +2 z terms are folded into the products as dual
    products with constant multipliers (-2/3, -1/3, 2/3, 1/3, 1/6), so that every output is a
    small combination of PRODUCTS (bounded, < 47 p) and never carries the input's size forward.
    Coefficient index = h 6 + jj 2 + k (w^(2 jj + h), Fp2 component k); 12 = the zero slot.
    Returns (rows, combine): rows[r] = (X, ybias, ypos, yneg, sbias, spos, sneg, kidx) for the 18
    product rows (0..11 dual products, 12..17 single), combine[o] = (pos, neg) [(slot, weight)]
    for the 12 output coefficients.  Checked against f12 squaring by tools/gen_dfp.py --check."""
    KIDX = {"M23": 0, "M13": 1, "P23": 2, "P13": 3, "P16": 4}
    pairs = [
        dict(a=(0, 1), b=(8, 9), zx=(0, 1), zy=(8, 9)),
        dict(a=(6, 7), b=(4, 5), zx=(2, 3), zy=(10, 11)),
        dict(a=(2, 3), b=(10, 11), zx=(4, 5), z2=(6, 7)),
    ]
    rows = []
    for p_, d in enumerate(pairs):
        a0, a1 = d["a"]
        b0, b1 = d["b"]
        x0, x1 = d["zx"]
        rows.append(([a0, a1], 1, [a0], [a1], 0, [x0], [], KIDX["M23"]))          # A0'
        rows.append(([a0], 0, [a1], [], 0, [x1], [], KIDX["M13"]))                 # A1'
        if p_ < 2:
            y0, y1 = d["zy"]
            rows.append(([a0, a1, b0, b1], 1, [a0, b0], [a1, b1], 1, [y0], [x0], KIDX["P23"]))  # C0'
            rows.append(([a0, b0], 0, [a1, b1], [], 1, [y1], [x1], KIDX["P13"]))                 # C1'
        else:
            z20, z21 = d["z2"]
            rows.append(([a0, a1, b0, b1], 1, [a0, b0], [a1, b1], 1, [z20, z21], [x0, x0], KIDX["P13"]))
            rows.append(([a0, b0], 0, [a1, b1], [], 1, [z21], [z20, x1, x1], KIDX["P16"]))
    for p_, d in enumerate(pairs):
        b0, b1 = d["b"]
        rows.append(([b0, b1], 1, [b0], [b1], 0, [], [], 255))   # B0
        rows.append(([b0], 0, [b1], [], 0, [], [], 255))          # B1

    def sl(p_):
        return dict(A0=4 * p_, A1=4 * p_ + 1, C0=4 * p_ + 2, C1=4 * p_ + 3, B0=12 + 2 * p_, B1=13 + 2 * p_)

    def t0(p_):
        s_ = sl(p_)
        return (([(s_["A0"], 3), (s_["B0"], 3)], [(s_["B1"], 6)]),
                ([(s_["A1"], 6), (s_["B0"], 3), (s_["B1"], 6)], []))

    def t1(p_):
        s_ = sl(p_)
        return (([(s_["C0"], 3)], [(s_["A0"], 3), (s_["B0"], 3)]),
                ([(s_["C1"], 6)], [(s_["A1"], 6), (s_["B1"], 6)]))

    def xt1(p_):
        s_ = sl(p_)
        return (([(s_["C0"], 3), (s_["A1"], 6), (s_["B1"], 6)], [(s_["A0"], 3), (s_["B0"], 3), (s_["C1"], 6)]),
                ([(s_["C0"], 3), (s_["C1"], 6)], [(s_["A0"], 3), (s_["B0"], 3), (s_["A1"], 6), (s_["B1"], 6)]))

    comb = [None] * 12
    comb[0], comb[1] = t0(0)
    comb[8], comb[9] = t1(0)
    comb[2], comb[3] = t0(1)
    comb[10], comb[11] = t1(1)
    comb[4], comb[5] = t0(2)
    comb[6], comb[7] = xt1(2)
    return rows, comb


def gs_check():
    """The plan against Fp12 squaring on cyclotomic elements (plain integers mod p)."""
    import random
    inv3, inv6 = pow(3, -1, P), pow(6, -1, P)
    kv = [(-2 * inv3) % P, (-inv3) % P, (2 * inv3) % P, inv3, inv6]
    rows, comb = gs_plan()
    xi = (1, 1)

    def f2m(a, b):
        return ((a[0] * b[0] - a[1] * b[1]) % P, (a[0] * b[1] + a[1] * b[0]) % P)

    def f12m(a, b):  # lists of 6 Fp2 coefficients of w^i, w^6 = xi
        t = [(0, 0)] * 11
        for i in range(6):
            for j in range(6):
                m = f2m(a[i], b[j])
                t[i + j] = ((t[i + j][0] + m[0]) % P, (t[i + j][1] + m[1]) % P)
        out = t[:6]
        for k_ in range(6, 11):
            m = f2m(t[k_], xi)
            out[k_ - 6] = ((out[k_ - 6][0] + m[0]) % P, (out[k_ - 6][1] + m[1]) % P)
        return out

    def to_c(x):
        c = [0] * 12
        for i in range(6):
            h, jj = i % 2, i // 2
            c[6 * h + 2 * jj], c[6 * h + 2 * jj + 1] = x[i]
        return c

    def f12pow(a, e):
        r_ = [(1, 0)] + [(0, 0)] * 5
        while e:
            if e & 1:
                r_ = f12m(r_, a)
            a = f12m(a, a)
            e >>= 1
        return r_

    rng = random.Random(7)
    f = [(rng.randrange(P), rng.randrange(P)) for _ in range(6)]
    g = f12pow(f, (P ** 6 - 1) * (P ** 2 + 1))  # cyclotomic
    for _ in range(3):
        c = to_c(g) + [0]
        prods = []
        for X, yb, yp, yn, sb, sp, sn, kidx in rows:
            v = sum(c[i] for i in X) * (sum(c[i] for i in yp) - sum(c[i] for i in yn))
            if kidx != 255:
                v += (sum(c[i] for i in sp) - sum(c[i] for i in sn)) * kv[kidx]
            prods.append(v % P)
        got = [(sum(prods[i] * w_ for i, w_ in pos) - sum(prods[i] * w_ for i, w_ in neg)) % P for pos, neg in comb]
        g = f12m(g, g)
        assert got == to_c(g)


# Fp2 arithmetic for the Frobenius constants: (a0, a1) = a0 + a1 u, u^2 = -1
def f2_mul(a, b):
    return ((a[0] * b[0] - a[1] * b[1]) % P, (a[0] * b[1] + a[1] * b[0]) % P)


def f2_pow(a, e):
    r = (1, 0)
    while e:
        if e & 1:
            r = f2_mul(r, a)
        a = f2_mul(a, a)
        e >>= 1
    return r


def f2_inv(a):
    n = pow(a[0] * a[0] + a[1] * a[1], P - 2, P)
    return (a[0] * n % P, -a[1] * n % P)


def main():
    pinv = (-pow(P, -1, R)) % R
    pl, pp = limbs(P), limbs(pinv)
    xi = (1, 1)
    frob1 = [f2_pow(xi, e * (P - 1) // 6) for e in range(6)]
    frob2 = [f2_pow(xi, e * (P * P - 1) // 6) for e in range(6)]
    assert all(f[1] == 0 for f in frob2)
    cx = f2_inv(f2_pow(xi, (P - 1) // 3))
    cy = f2_inv(f2_pow(xi, (P - 1) // 2))
    psi2x = f2_mul((cx[0], -cx[1] % P), cx)
    psi2y = f2_mul((cy[0], -cy[1] % P), cy)
    assert cx[0] == 0 and psi2x[1] == 0 and psi2y[1] == 0
    consts = {
        "P": limbs(P),
        "CIN": limbs(pow(2, 2 * N * W - 384, P)),   # engine form (x 2^384) -> x 2^448
        "COUT": limbs(pow(2, 384, P)),              # x 2^448 -> x 2^384
        "ONE": limbs(mont(1)),
        # subtraction biases: R1 of the Fp12 product subtracts <= 6 products (< 1.0001 p,
        # limbs < 2^28 + 2^9); R2 <= 2 R1 values (< 14.001 p, limbs < 2^28 + 16); NEG negates
        # one coefficient (< 128 p, limbs < 2^28 + 2^9)
        "BIAS_R1": rebalanced(8 * P, 7),
        "BIAS_R2": rebalanced(32 * P, 3),
        "BIAS_NEG": rebalanced(128 * P, 2),
        # the squaring's (x0 - x1) operands subtract <= 4 coefficients (< 128 p each, limbs
        # < 2^28 + 2^9): 1024 p with 5 units borrowed per limb
        "BIAS_SQ": rebalanced(1024 * P, 5),
        # cyclotomic squaring operands: Y subtracts <= 2 coefficients, S <= 3 (< 128 p each; 2x
        # headroom, as BIAS_SQ, so that the unborrowed top limb never goes negative)
        "BIAS_GY": rebalanced(512 * P, 3),
        "BIAS_GS": rebalanced(1024 * P, 4),
        # the easy part's inversion (bls_w12d.h inv_fp): inverse_words(x 2^384) = x^-1 2^-384,
        # times 2^1280 / 2^448 -> x^-1 2^448
        "INVFIX": limbs(pow(2, 1280, P)),
        # G2 endomorphisms (bls_w4.h): psi = (conj(x) cx, conj(y) cy) with cx = (0, PSI_CX1);
        # psi^2 = (x PSI2_CX, y PSI2_CY), both in Fp
        "PSI_CX1": limbs(mont(cx[1])),
        "PSI_CY0": limbs(mont(cy[0])),
        "PSI_CY1": limbs(mont(cy[1])),
        "PSI2_CX": limbs(mont(psi2x[0])),
        "PSI2_CY": limbs(mont(psi2y[0])),
    }
    out = []
    w = out.append
    w("// GENERATED by tools/gen_dfp.py -- do not edit.")
    w("// Row-distributed Fp (bls_dfp.h): 16 limbs of 28 bits, one per lane of a DPP row,")
    w("// Montgomery form with R = 2^448.")
    w("#pragma once")
    w("#include <stdint.h>")
    w("namespace gbls { namespace dfp {")
    w("constexpr uint64_t X_ABS = 0x%016xull;" % X_ABS)
    pre, r1, r2 = w12d_plan()
    w("// Row-distributed Fp12 product (bls_w12d.h): per-row operand / term plans")
    w("constexpr int W12D_ZERO = 72, W12D_NSLOT = 73;")
    w("__constant__ uint8_t W12D_PRE[54][8] = {")
    for row in pre:
        w("  {%s}," % ", ".join(str(v) for v in row))
    w("};")
    w("// R1: 6 positive then 6 negative product slots")
    w("__constant__ uint8_t W12D_R1[18][12] = {")
    for row in r1:
        w("  {%s}," % ", ".join(str(v) for v in row))
    w("};")
    w("// R2: 3 positive then 2 negative R1 slots")
    w("__constant__ uint8_t W12D_R2[12][5] = {")
    for row in r2:
        w("  {%s}," % ", ".join(str(v) for v in row))
    w("};")
    sl, srp, srn, sr1, sr2 = w12d_sqr_plan()
    w("// Row-distributed Fp12 squaring (bls_w12d.h sqr): lhs / rhs+ / rhs- coefficient sets, R1, R2")
    w("__constant__ uint8_t W12S_L[36][8] = {")
    for row in sl:
        w("  {%s}," % ", ".join(str(v) for v in row))
    w("};")
    w("__constant__ uint8_t W12S_RP[36][4] = {")
    for row in srp:
        w("  {%s}," % ", ".join(str(v) for v in row))
    w("};")
    w("__constant__ uint8_t W12S_RN[36][4] = {")
    for row in srn:
        w("  {%s}," % ", ".join(str(v) for v in row))
    w("};")
    w("__constant__ uint8_t W12S_R1[18][12] = {")
    for row in sr1:
        w("  {%s}," % ", ".join(str(v) for v in row))
    w("};")
    w("__constant__ uint8_t W12S_R2[12][5] = {")
    for row in sr2:
        w("  {%s}," % ", ".join(str(v) for v in row))
    w("};")
    gs_check()
    grows, gcomb = gs_plan()
    w("// Granger-Scott cyclotomic squaring (bls_w12d.h cyc_sqr; tools/gen_dfp.py gs_plan), packed per")
    w("// row.  Product rows 0..17, word 0: X coefficients (4 nibbles), Y positive (2), Y negative (2);")
    w("// word 1: S positive (2 nibbles), S negative (3), bit 20 Y bias, bit 21 S bias, bits 22..24 the")
    w("// K_GS index (7: a single product).  Coefficient 12 = zero.  Combine rows 0..11: 4 positive then")
    w("// 4 negative terms, one byte each: product slot (bits 0..6; W12D_ZERO = none), bit 7 = weight 2")
    w("// (else 1); the output is 3 (BIAS_R1 + positive - negative).")
    pad = lambda l, n, z: list(l) + [z] * (n - len(l))
    w("__constant__ uint32_t W12G_ROW[18][2] = {")
    for X, yb, yp, yn, sb, sp, sn, kidx in grows:
        nib = pad(X, 4, 12) + pad(yp, 2, 12) + pad(yn, 2, 12)
        w0 = sum(v << (4 * k) for k, v in enumerate(nib))
        nib = pad(sp, 2, 12) + pad(sn, 3, 12)
        w1 = sum(v << (4 * k) for k, v in enumerate(nib)) | yb << 20 | sb << 21 | (7 if kidx == 255 else kidx) << 22
        w("  {0x%08xu, 0x%08xu}," % (w0, w1))
    w("};")
    w("__constant__ uint32_t W12G_COMB[12][2] = {")
    zero_slot = 72
    for pos, neg in gcomb:
        by = []
        for t_ in pad(pos, 4, None) + pad(neg, 4, None):
            if t_ is None:
                by.append(zero_slot)
            else:
                assert t_[1] in (3, 6)
                by.append(t_[0] | (128 if t_[1] == 6 else 0))
        w("  {0x%08xu, 0x%08xu}," % (sum(v << (8 * k) for k, v in enumerate(by[:4])), sum(v << (8 * k) for k, v in enumerate(by[4:]))))
    w("};")
    inv3, inv6 = pow(3, -1, P), pow(6, -1, P)
    w("// the folded z terms' multipliers -2/3, -1/3, 2/3, 1/3, 1/6 (Montgomery row form)")
    w("__constant__ uint32_t K_GS[5][16] = {")
    for v in [(-2 * inv3) % P, (-inv3) % P, (2 * inv3) % P, inv3, inv6]:
        w("  {%s}," % ", ".join("0x%08xu" % x for x in limbs(mont(v))))
    w("};")
    w("// Frobenius constants by exponent e of w: FROB1[e] = (c0, c1) of xi^(e (p - 1) / 6),")
    w("// FROB2[e] = xi^(e (p^2 - 1) / 6) (in Fp); e = 0 is one")
    one = limbs(mont(1))
    w("__constant__ uint32_t K_FROB1[6][2][16] = {")
    for e in range(6):
        c0 = one if e == 0 else limbs(mont(frob1[e][0]))
        c1 = [0] * 16 if e == 0 else limbs(mont(frob1[e][1]))
        w("  {{%s}, {%s}}," % (", ".join("0x%07xu" % v for v in c0), ", ".join("0x%07xu" % v for v in c1)))
    w("};")
    w("__constant__ uint32_t K_FROB2[6][16] = {")
    for e in range(6):
        c = one if e == 0 else limbs(mont(frob2[e][0]))
        w("  {%s}," % ", ".join("0x%07xu" % v for v in c))
    w("};")
    w("// wave-uniform limbs of p and p' = -p^-1 mod 2^448 (compile-time constants: SGPR operands)")
    w("constexpr uint32_t K_P_U[16] = {%s};" % ", ".join("0x%07xu" % v for v in pl))
    w("constexpr uint32_t K_PINV_U[16] = {%s};" % ", ".join("0x%07xu" % v for v in pp))
    w("// per-lane limbs of constants: K_<NAME>[j] = limb j")
    for name, l in consts.items():
        w("__constant__ uint32_t K_%s[16] = {%s};" % (name, ", ".join("0x%08xu" % v for v in l)))
    w("// subtraction biases 2^k p (k = 1..10) for bls_w4.h, lower limbs pre-borrowed (2 units)")
    w("__constant__ uint32_t K_BIASK[10][16] = {")
    for kk in range(1, 11):
        w("  {%s}," % ", ".join("0x%08xu" % v for v in rebalanced((1 << kk) * P, 2)))
    w("};")
    w("}}  // namespace gbls::dfp")
    print("\n".join(out))


if __name__ == "__main__":
    main()
