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
    print("\n".join(out))


if __name__ == "__main__":
    main()
