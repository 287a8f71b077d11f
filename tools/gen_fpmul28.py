#!/usr/bin/env python3
"""Generate grandine_amd/csrc/bls_fpmul28_gen.h: the gfx950 radix-2^28 Montgomery products of
bls_field28.h (14 limbs of 28 bits, R = 2^392).

Same product-scanning schedule as tools/gen_fpmul.py, but a column's terms are < 2^58 and
at most 42 of them meet in one column, so the 64-bit accumulator needs no carry word: ONE
v_mad_u64_u32 per term.  Each column is one `asm volatile` statement (split every
MAX_TERMS terms), which keeps the products in program order (plain C lets the compiler
reassociate the column sums and run many products at once, which spilled k_ml_group28 to
scratch).

fe_mul4_dev / fe_mul6_dev: the sum of four / SIX products in one reduction -- one output coordinate of the lazy
sparse Miller product (bls_field28.h fe12_mul_034_lazy: every Fp12 coefficient of f * line is
a sum of three Fp2 products, i.e. six Fp products per Fp coordinate).  Bound: with one operand
of each pair normalized (limbs < 2^28) and the other < 2^29, a column holds at most
14 * (6 * 2^57) + 14 * 2^56 < 2^63.3 (no overflow of the 64-bit accumulator).

Run:  python tools/gen_fpmul28.py > grandine_amd/csrc/bls_fpmul28_gen.h
"""

N = 14


MAX_TERMS = 28
# GEN28_SPLIT=1: every column of >= 4 terms as two interleaved accumulator chains.  Measured r05
# (GBLS_LIB A/B on C2): 4.17M vs 4.19-4.24M sets/s with the radix-2^28 lanes off, 4.03M vs 4.26M
# with them on; +4.5 % instructions, VALU busy unchanged -- the single chain is not the stall.
# The generated header keeps the single chain (SPLIT off).
import os  # noqa: E402
SPLIT = os.environ.get("GEN28_SPLIT", "0") == "1"


def emit_asm(terms):
    if len(terms) > MAX_TERMS:
        return "\n".join(emit_asm(terms[i:i + MAX_TERMS]) for i in range(0, len(terms), MAX_TERMS))
    lines, ops = [], []
    for x, y in terms:
        xi = len(ops) + 1
        ops.append(("v", x))
        if x == y:  # a diagonal term: one operand, used twice
            lines.append("v_mad_u64_u32 %%0, vcc, %%%d, %%%d, %%0" % (xi, xi))
            continue
        yi = len(ops) + 1
        ops.append(("s" if y.startswith("P") else "v", y))
        lines.append("v_mad_u64_u32 %%0, vcc, %%%d, %%%d, %%0" % (xi, yi))
    body = "\\n\\t".join(lines)
    inputs = ", ".join('"%s"(%s)' % (c, v) for c, v in ops)
    return '    asm volatile("%s"\n        : "+&v"(acc)\n        : %s\n        : "vcc");' % (body, inputs)


def emit_asm2(terms):
    """The terms alternate between two accumulators (acc, acc2) inside ONE asm statement: two
    independent v_mad_u64_u32 chains, so consecutive products do not wait on each other."""
    if len(terms) > MAX_TERMS:
        return "\n".join(emit_asm2(terms[i:i + MAX_TERMS]) for i in range(0, len(terms), MAX_TERMS))
    lines, ops = [], []
    for n, (x, y) in enumerate(terms):
        xi = len(ops) + 2
        ops.append(("v", x))
        yi = len(ops) + 2
        ops.append(("s" if y.startswith("P") else "v", y))
        a = n % 2
        lines.append("v_mad_u64_u32 %%%d, vcc, %%%d, %%%d, %%%d" % (a, xi, yi, a))
    body = "\\n\\t".join(lines)
    inputs = ", ".join('"%s"(%s)' % (c, v) for c, v in ops)
    return '    asm volatile("%s"\n        : "+&v"(acc), "+&v"(acc2)\n        : %s\n        : "vcc");' % (body, inputs)


def emit_column(terms):
    """One column's terms: a single chain, or (SPLIT) two chains summed at the end."""
    if SPLIT and len(terms) >= 4:
        return "    acc2 = 0;\n" + emit_asm2(terms) + "\n    acc += acc2;"
    return emit_asm(terms)


def emit_product(w, name, params, pairs):
    w("__device__ __forceinline__ void %s(%s) {" % (name, params))
    for j in range(N):
        w("  const uint32_t P%d = %s;" % (j, "kP28[%d]" % j))
    w("  uint32_t " + ", ".join("m%d" % j for j in range(N)) + ";")
    w("  uint32_t t[14];")
    w("  uint64_t acc = 0;")
    if SPLIT:
        w("  uint64_t acc2;")
    for k in range(2 * N - 1):
        ab = [("%s.l[%d]" % (x, i), "%s.l[%d]" % (y, k - i)) for (x, y) in pairs for i in range(N)
              if 0 <= k - i < N]
        mp = [("m%d" % i, "P%d" % (k - i)) for i in range(N) if i < k and 0 <= k - i < N]
        w("  {  // column %d" % k)
        if k < N:
            if ab + mp:
                w(emit_column(ab + mp))
            w("    m%d = ((uint32_t)acc * kPinv) & kMask;" % k)
            w(emit_asm([("m%d" % k, "P0")]))
        else:
            w(emit_column(ab + mp))
            w("    t[%d] = (uint32_t)acc & kMask;" % (k - N))
        w("    acc >>= 28;")
        w("  }")
    w("  t[13] = (uint32_t)acc;")
    w("#pragma unroll")
    w("  for (int i = 0; i < 14; i++) r.l[i] = t[i];")
    w("}")


def emit_square(w, name):
    """r = a^2 / 2^392: the cross terms once against the doubled limbs (d = 2a, limbs < 2^30),
    the diagonal once: 105 product terms instead of 196 before the 196 of the reduction.
    Column bound: 7 cross terms < 2^59 + a diagonal < 2^58 + 14 reduction terms < 2^56 < 2^63."""
    w("__device__ __forceinline__ void %s(fe &r, const fe &a) {" % name)
    for j in range(N):
        w("  const uint32_t P%d = %s;" % (j, "kP28[%d]" % j))
    w("  uint32_t d[14];")
    w("#pragma unroll")
    w("  for (int i = 0; i < 14; i++) d[i] = a.l[i] << 1;")
    w("  uint32_t " + ", ".join("m%d" % j for j in range(N)) + ";")
    w("  uint32_t t[14];")
    w("  uint64_t acc = 0;")
    if SPLIT:
        w("  uint64_t acc2;")
    for k in range(2 * N - 1):
        ab = [("d[%d]" % i, "a.l[%d]" % (k - i)) for i in range(N) if i < k - i < N]
        if k % 2 == 0 and k // 2 < N:
            ab.append(("a.l[%d]" % (k // 2), "a.l[%d]" % (k // 2)))
        mp = [("m%d" % i, "P%d" % (k - i)) for i in range(N) if i < k and 0 <= k - i < N]
        w("  {  // column %d" % k)
        if k < N:
            if ab + mp:
                w(emit_column(ab + mp))
            w("    m%d = ((uint32_t)acc * kPinv) & kMask;" % k)
            w(emit_asm([("m%d" % k, "P0")]))
        else:
            w(emit_column(ab + mp))
            w("    t[%d] = (uint32_t)acc & kMask;" % (k - N))
        w("    acc >>= 28;")
        w("  }")
    w("  t[13] = (uint32_t)acc;")
    w("#pragma unroll")
    w("  for (int i = 0; i < 14; i++) r.l[i] = t[i];")
    w("}")


P_INT = 0x1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaaab
# c0 = sum x_q.c0 u_q.c0 - sum x_q.c1 u_q.c1 can be negative: BIAS_KARA (a multiple of p^2, so
# the value is unchanged mod p) is added column by column; 17 p^2 exceeds the largest
# sum x_q.c1 u_q.c1 of the sparse Miller product (3 x 1.1p x 5.1p)
BIAS_KARA = 17 * P_INT * P_INT


def emit_kara3(w, name):
    """r = x_0 u_0 + x_1 u_1 + x_2 u_2 over Fp2 = Fp[i]/(i^2 + 1), Karatsuba per Fp2 product and
    ONE Montgomery reduction per output coordinate (k_ml_group28's sparse product, r06):
        A = sum x_q.c0 u_q.c0,  B = sum x_q.c1 u_q.c1,  C = sum (x_q.c0 + x_q.c1)(u_q.c0 + u_q.c1)
        r.c0 = (A - B + BIAS) / 2^392,   r.c1 = (C - A - B) / 2^392
    9 products of 196 terms instead of 12 (fe_mul6_dev twice).  Per column k the three sums
    are formed apart (A in a, B in b, C straight into acc1), then acc0 += a - b + BIAS_k (signed:
    a column of A - B can be negative; |A_k - B_k| < 42 x 2^56) and acc1 -= a + b (C_k - A_k -
    B_k is the column of the cross terms x0 u1 + x1 u0 >= 0, < 84 x 2^56); the sums' operands
    have limbs < 2^29, so a column of C is < 42 x 2^58 < 2^63.4 (no overflow of the unsigned
    64-bit accumulator).  Inputs: x_q, u_q normalized (limbs < 2^28); values < 1.1 p (x) and
    < 5.1 p (u); xs_q / us_q their limbwise sums.  Outputs < 1.03 p, normalized."""
    bias = [(BIAS_KARA >> (28 * k)) & 0xfffffff for k in range(28)]
    assert BIAS_KARA >> (28 * 28) == 0
    Q = 3
    params = ["fe &r0", "fe &r1"]
    for q in range(Q):
        params += ["const fe &x%da" % q, "const fe &x%db" % q, "const fe &u%da" % q, "const fe &u%db" % q,
                   "const fe &u%ds" % q]
    w("__device__ __forceinline__ void %s(%s) {" % (name, ", ".join(params)))
    for j in range(N):
        w("  const uint32_t P%d = kP28[%d];" % (j, j))
    for q in range(Q):
        w("  uint32_t xs%d[14];" % q)
        w("#pragma unroll")
        w("  for (int i = 0; i < 14; i++) xs%d[i] = x%da.l[i] + x%db.l[i];" % (q, q, q))
    w("  uint32_t " + ", ".join("m%d_%d" % (h, j) for h in range(2) for j in range(N)) + ";")
    w("  uint32_t t0[14], t1[14];")
    w("  int64_t acc0 = 0;")
    w("  uint64_t acc1 = 0;")

    def asm_into(var, terms, fresh):
        # var (+)= sum of terms; fresh: the first mad adds 0 (the inline constant)
        out = []
        for c in range(0, len(terms), MAX_TERMS):
            chunk = terms[c:c + MAX_TERMS]
            lines, ops = [], []
            for n_, (x, y) in enumerate(chunk):
                xi = len(ops) + 1
                ops.append(("v", x))
                yi = len(ops) + 1
                ops.append(("s" if y.startswith("P") else "v", y))
                src2 = "0" if (fresh and c == 0 and n_ == 0) else "%0"
                lines.append("v_mad_u64_u32 %%0, vcc, %%%d, %%%d, %s" % (xi, yi, src2))
            body = "\\n\\t".join(lines)
            inputs = ", ".join('"%s"(%s)' % (cc, v) for cc, v in ops)
            cons = '"=&v"' if (fresh and c == 0) else '"+&v"'
            out.append('    asm volatile("%s"\n        : %s(%s)\n        : %s\n        : "vcc");'
                       % (body, cons, var, inputs))
        return "\n".join(out)

    for k in range(2 * N - 1):
        idx = [(i, k - i) for i in range(N) if 0 <= k - i < N]
        A = [("x%da.l[%d]" % (q, i), "u%da.l[%d]" % (q, j)) for q in range(Q) for i, j in idx]
        B = [("x%db.l[%d]" % (q, i), "u%db.l[%d]" % (q, j)) for q in range(Q) for i, j in idx]
        C = [("xs%d[%d]" % (q, i), "u%ds.l[%d]" % (q, j)) for q in range(Q) for i, j in idx]
        w("  {  // column %d" % k)
        w("    uint64_t a, b;")
        w(asm_into("a", A, True))
        w(asm_into("b", B, True))
        w(asm_into("acc1", C, False))
        w("    acc0 += (int64_t)(a - b) + (int64_t)0x%xll;" % bias[k])
        w("    acc1 -= a + b;")
        for h, acc in ((0, "acc0"), (1, "acc1")):
            mp = [("m%d_%d" % (h, i), "P%d" % (k - i)) for i in range(N) if i < k and 0 <= k - i < N]
            if mp:
                w(asm_into(acc, mp, False))
            if k < N:
                w("    m%d_%d = ((uint32_t)%s * kPinv) & kMask;" % (h, k, acc))
                w(asm_into(acc, [("m%d_%d" % (h, k), "P0")], False))
            else:
                w("    t%d[%d] = (uint32_t)%s & kMask;" % (h, k - N, acc))
        w("    acc0 >>= 28;  // arithmetic: a column of c0 may be negative")
        w("    acc1 >>= 28;")
        w("  }")
    w("  t0[13] = (uint32_t)acc0 + 0x%xu;  // the bias's top limb" % bias[27])
    w("  t1[13] = (uint32_t)acc1;")
    w("#pragma unroll")
    w("  for (int i = 0; i < 14; i++) r0.l[i] = t0[i], r1.l[i] = t1[i];")
    w("}")


def main():
    out = []
    w = out.append
    w("// GENERATED by tools/gen_fpmul28.py -- do not edit.")
    w("// Device radix-2^28 Montgomery products (bls_field28.h): one asm statement per column,")
    w("// one v_mad_u64_u32 per term.  fe_mul_dev: a b / 2^392; fe_mul2_dev: (a b + c d) / 2^392.")
    w("#pragma once")
    w("// included from bls_field28.h inside namespace gbls::r28, device compilation only")
    emit_product(w, "fe_mul_dev", "fe &r, const fe &a, const fe &b", (("a", "b"),))
    emit_product(w, "fe_mul2_dev", "fe &r, const fe &a, const fe &b, const fe &c, const fe &d",
                 (("a", "b"), ("c", "d")))
    emit_square(w, "fe_sqr_dev")
    names = [("x%d" % q, "y%d" % q) for q in range(4)]
    emit_product(w, "fe_mul4_dev", "fe &r, " + ", ".join("const fe &%s, const fe &%s" % xy for xy in names),
                 tuple(names))
    names = [("x%d" % q, "y%d" % q) for q in range(6)]
    emit_product(w, "fe_mul6_dev", "fe &r, " + ", ".join("const fe &%s, const fe &%s" % xy for xy in names),
                 tuple(names))
    emit_kara3(w, "fe2_mul3k_dev")
    print("\n".join(out))


if __name__ == "__main__":
    main()
