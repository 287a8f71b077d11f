// G1 (E: y^2 = x^3 + 4 over Fp) and G2 (E': y^2 = x^3 + 4(1+u) over Fp2) arithmetic.
//
// Replaces blst's POINTonE1 / POINTonE2 layer used by PublicKey::aggregate
// (bls/src/public_key.rs:34-55), decompression (public_key.rs:16-31,
// signature.rs:36-45), compression (public_key.rs:9-14, signature.rs:29-34) and the
// 64-bit random-scalar multiplications inside verify_multiple_aggregate_signatures
// (signature.rs:117-126).  Jacobian coordinates (x = X/Z^2, y = Y/Z^3), Z = 0 is the
// point at infinity; affine infinity is all-zero limbs, as in blst.
#pragma once
#include "bls_field.h"

namespace gbls {

// ----- overload set so one template serves Fp and Fp2 curves
HD void f_add(fp &r, const fp &a, const fp &b) { fp_add(r, a, b); }
HD void f_sub(fp &r, const fp &a, const fp &b) { fp_sub(r, a, b); }
HD void f_mul(fp &r, const fp &a, const fp &b) { fp_mul(r, a, b); }
HD void f_sqr(fp &r, const fp &a) { fp_sqr(r, a); }
HD void f_neg(fp &r, const fp &a) { fp_neg(r, a); }
HD void f_dbl(fp &r, const fp &a) { fp_add(r, a, a); }
HD bool f_is_zero(const fp &a) { return fp_is_zero(a); }
HD bool f_eq(const fp &a, const fp &b) { return fp_eq(a, b); }
HD void f_one(fp &r) { fp_one(r); }
HD void f_zero(fp &r) { fp_zero(r); }
HD void f_inv(fp &r, const fp &a) { fp_inv(r, a); }
HD void f_add(fp2 &r, const fp2 &a, const fp2 &b) { fp2_add(r, a, b); }
HD void f_sub(fp2 &r, const fp2 &a, const fp2 &b) { fp2_sub(r, a, b); }
HD void f_mul(fp2 &r, const fp2 &a, const fp2 &b) { fp2_mul(r, a, b); }
HD void f_sqr(fp2 &r, const fp2 &a) { fp2_sqr(r, a); }
HD void f_neg(fp2 &r, const fp2 &a) { fp2_neg(r, a); }
HD void f_dbl(fp2 &r, const fp2 &a) { fp2_add(r, a, a); }
HD bool f_is_zero(const fp2 &a) { return fp2_is_zero(a); }
HD bool f_eq(const fp2 &a, const fp2 &b) { return fp2_eq(a, b); }
HD void f_one(fp2 &r) { fp2_one(r); }
HD void f_zero(fp2 &r) { fp2_zero(r); }
HD void f_inv(fp2 &r, const fp2 &a) { fp2_inv(r, a); }

template <class F>
struct jac {
  F x, y, z;
};
template <class F>
struct aff {
  F x, y;
};
typedef jac<fp> g1j;
typedef jac<fp2> g2j;
typedef aff<fp> g1a;
typedef aff<fp2> g2a;

template <class F>
HD bool aff_is_inf(const aff<F> &a) {
  return f_is_zero(a.x) && f_is_zero(a.y);
}
template <class F>
HD bool jac_is_inf(const jac<F> &a) {
  return f_is_zero(a.z);
}
template <class F>
HD void jac_set_inf(jac<F> &r) {
  f_one(r.x);
  f_one(r.y);
  f_zero(r.z);
}
template <class F>
HD void jac_from_aff(jac<F> &r, const aff<F> &a) {
  r.x = a.x;
  r.y = a.y;
  if (aff_is_inf(a))
    f_zero(r.z);
  else
    f_one(r.z);
}
template <class F>
HD void jac_neg(jac<F> &r, const jac<F> &a) {
  r.x = a.x;
  f_neg(r.y, a.y);
  r.z = a.z;
}

// The formulas below are written in liveness order: every input coordinate is consumed
// as early as possible, so that (with the field products kept in program order, see
// tools/gen_fpmul.py) a G2 point operation needs few live Fp2 temporaries.

// dbl-2009-l (a = 0): 2M + 5S.  r may alias p.
template <class F>
HD void jac_dbl(jac<F> &r, const jac<F> &p) {
  F A, B, C, t;
  f_mul(t, p.y, p.z);
  f_sqr(A, p.x);
  f_sqr(B, p.y);
  f_add(C, p.x, B);  // X + B
  f_dbl(r.z, t);     // Z3 = 2YZ   (p.y, p.z dead)
  f_sqr(t, C);       // (X + B)^2  (p.x dead)
  f_sqr(C, B);       // C = B^2    (B dead)
  f_sub(t, t, A);
  f_sub(t, t, C);
  f_dbl(B, t);       // D = 2((X+B)^2 - A - C)
  f_dbl(t, A);
  f_add(A, t, A);    // E = 3A
  f_sqr(t, A);       // F = E^2
  f_sub(t, t, B);
  f_sub(r.x, t, B);  // X3 = F - 2D
  f_sub(t, B, r.x);
  f_mul(t, A, t);    // E (D - X3)
  f_dbl(C, C);
  f_dbl(C, C);
  f_dbl(C, C);
  f_sub(r.y, t, C);  // Y3 = E (D - X3) - 8C
}

// add-2007-bl, r = a + b.  r may alias a (NOT b): the degenerate cases (a == +-b)
// recompute from b, so a's coordinates can be consumed early.
template <class F>
HD void jac_add(jac<F> &r, const jac<F> &a, const jac<F> &b) {
  if (jac_is_inf(b)) {
    r = a;
    return;
  }
  if (jac_is_inf(a)) {
    r = b;
    return;
  }
  F z1z1, z2z2, u1, u2, s1, s2, t;
  f_sqr(z1z1, a.z);
  f_sqr(z2z2, b.z);
  f_mul(u1, a.x, z2z2);
  f_mul(u2, b.x, z1z1);
  f_mul(s1, a.y, b.z);
  f_mul(s1, s1, z2z2);
  f_mul(s2, b.y, a.z);
  f_mul(s2, s2, z1z1);
  f_add(t, a.z, b.z);
  f_sqr(t, t);
  f_sub(t, t, z1z1);
  f_sub(t, t, z2z2);  // 2 Z1 Z2            (z1z1, z2z2, a.* dead)
  f_sub(u2, u2, u1);  // H
  f_sub(s2, s2, s1);
  f_dbl(s2, s2);      // r = 2 (S2 - S1)
  if (f_is_zero(u2)) {
    if (f_is_zero(s2))
      jac_dbl(r, b);
    else
      jac_set_inf(r);
    return;
  }
  f_mul(r.z, t, u2);  // Z3 = 2 Z1 Z2 H
  f_dbl(t, u2);
  f_sqr(t, t);        // I = (2H)^2
  f_mul(u2, u2, t);   // J = H I
  f_mul(u1, u1, t);   // V = U1 I
  f_sqr(t, s2);
  f_sub(t, t, u2);
  f_sub(t, t, u1);
  f_sub(r.x, t, u1);  // X3 = r^2 - J - 2V
  f_sub(t, u1, r.x);
  f_mul(t, s2, t);    // r (V - X3)
  f_mul(s1, s1, u2);
  f_dbl(s1, s1);      // 2 S1 J
  f_sub(r.y, t, s1);
}

// madd-2007-bl: r = a + b for b affine.  r may alias a.
template <class F>
HD void jac_add_aff(jac<F> &r, const jac<F> &a, const aff<F> &b) {
  if (aff_is_inf(b)) {
    r = a;
    return;
  }
  if (jac_is_inf(a)) {
    jac_from_aff(r, b);
    return;
  }
  F z1z1, u2, s2, t, hh;
  f_sqr(z1z1, a.z);
  f_mul(u2, b.x, z1z1);
  f_mul(s2, b.y, a.z);
  f_mul(s2, s2, z1z1);
  f_sub(u2, u2, a.x);  // H
  f_sub(s2, s2, a.y);
  f_dbl(s2, s2);       // r = 2 (S2 - Y1)
  if (f_is_zero(u2)) {
    if (f_is_zero(s2)) {
      jac<F> bj;
      jac_from_aff(bj, b);
      jac_dbl(r, bj);
    } else {
      jac_set_inf(r);
    }
    return;
  }
  f_add(t, a.z, u2);
  f_sqr(t, t);
  f_sub(t, t, z1z1);   // (Z1 + H)^2 - Z1Z1        (z1z1 dead)
  f_sqr(hh, u2);
  f_sub(r.z, t, hh);   // Z3 = (Z1 + H)^2 - Z1Z1 - HH   (a.z dead)
  f_dbl(hh, hh);
  f_dbl(hh, hh);       // I = 4 HH
  f_mul(z1z1, a.x, hh);  // V = X1 I
  f_mul(hh, u2, hh);     // J = H I
  f_mul(t, a.y, hh);
  f_dbl(u2, t);          // 2 Y1 J                  (a.x, a.y dead)
  f_sqr(t, s2);
  f_sub(t, t, hh);
  f_sub(t, t, z1z1);
  f_sub(r.x, t, z1z1);   // X3 = r^2 - J - 2V
  f_sub(t, z1z1, r.x);
  f_mul(t, s2, t);
  f_sub(r.y, t, u2);     // Y3 = r (V - X3) - 2 Y1 J
}

// No early return for infinity: Z = 0 inverts to 0 (fp_inv's loop ends at once) and the
// result is then zeroed by a select, so the point at infinity maps to (0, 0), the all-zero
// affine encoding.  (The early return made the compiler keep the output in scratch memory:
// 92 B per lane in every G2 kernel that ends with an affine conversion.)
template <class F>
HD void jac_to_aff(aff<F> &r, const jac<F> &p) {
  const bool inf = jac_is_inf(p);
  F zi, zi2, zi3;
  f_inv(zi, p.z);
  f_sqr(zi2, zi);
  f_mul(zi3, zi2, zi);
  f_mul(r.x, p.x, zi2);
  f_mul(r.y, p.y, zi3);
  if (inf) {
    f_zero(r.x);
    f_zero(r.y);
  }
}

// Jacobian equality without inversion: X1 Z2^2 == X2 Z1^2 and Y1 Z2^3 == Y2 Z1^3
template <class F>
HD bool jac_eq(const jac<F> &p, const jac<F> &q) {
  bool pi = jac_is_inf(p), qi = jac_is_inf(q);
  if (pi || qi) return pi && qi;
  F z1z1, z2z2, a, b;
  f_sqr(z1z1, p.z);
  f_sqr(z2z2, q.z);
  f_mul(a, p.x, z2z2);
  f_mul(b, q.x, z1z1);
  if (!f_eq(a, b)) return false;
  f_mul(a, p.y, q.z);
  f_mul(a, a, z2z2);
  f_mul(b, q.y, p.z);
  f_mul(b, b, z1z1);
  return f_eq(a, b);
}

// [k]P for an affine base and a 64-bit scalar, MSB-first double-and-add.
template <class F>
HD void mul_u64(jac<F> &r, const aff<F> &base, uint64_t k) {
  jac<F> acc;
  jac_set_inf(acc);
  if (k == 0 || aff_is_inf(base)) {
    r = acc;
    return;
  }
  int top = 63;
  while (!((k >> top) & 1)) top--;
  jac_from_aff(acc, base);
  for (int i = top - 1; i >= 0; i--) {
    jac_dbl(acc, acc);
    if ((k >> i) & 1) jac_add_aff(acc, acc, base);
  }
  r = acc;
}

HD void g1j_sel(g1j &r, bool c, const g1j &a, const g1j &b) {  // r = c ? b : a
  fp_sel(r.x, c, a.x, b.x);
  fp_sel(r.y, c, a.y, b.y);
  fp_sel(r.z, c, a.z, b.z);
}
// [k]P for an affine G1 base and a 64-bit scalar: signed 3-bit digits d_i in [-3, 4]
// (k = sum d_i 8^i, 22 digits) over the table {P, 2P, 3P, 4P}, 65 doublings + 22 Jacobian
// additions whatever k is.  Every lane runs the same instructions (the table entry and
// a zero digit are selects), so a wave of lanes with different scalars does not pay
// for both sides of every bit, as mul_u64's double-and-add does (63 doublings + 63 mixed
// additions per wave): 807 Fp products against 1134.
HD void g1_mul_u64_w3(g1j &r, const g1a &base, uint64_t k) {
  g1j t0, t1, t2, t3;
  jac_from_aff(t0, base);
  jac_dbl(t1, t0);
  jac_add(t2, t1, t0);
  jac_dbl(t3, t1);
  // carry into each window (LSB first), so the MSB-first loop can form its digit
  uint32_t cmask = 0, carry = 0;
#pragma unroll
  for (int i = 0; i < 22; i++) {
    cmask |= carry << i;
    carry = ((uint32_t)((k >> (3 * i)) & 7u) + carry) > 4;  // 3 i <= 63
  }
  g1j acc;
  jac_set_inf(acc);
  const uint32_t top = (uint32_t)(k >> 63) + (cmask >> 21);  // top digit in [0, 2]
  g1j_sel(acc, top == 1, acc, t0);
  g1j_sel(acc, top == 2, acc, t1);
#pragma unroll 1
  for (int i = 20; i >= 0; i--) {
    jac_dbl(acc, acc);
    jac_dbl(acc, acc);
    jac_dbl(acc, acc);
    int v = (int)((k >> (3 * i)) & 7u) + (int)((cmask >> i) & 1u);
    if (v > 4) v -= 8;
    const uint32_t m = (uint32_t)(v < 0 ? -v : v);
    g1j q = t0, s;
    g1j_sel(q, m == 2, q, t1);
    g1j_sel(q, m == 3, q, t2);
    g1j_sel(q, m == 4, q, t3);
    fp ny;
    fp_neg(ny, q.y);
    fp_sel(q.y, v < 0, q.y, ny);
    jac_add(s, acc, q);
    g1j_sel(acc, m != 0, acc, s);
  }
  r = acc;
}

// [|x|]P for a Jacobian point (|x| = 0xd201000000010000, 6 set bits) -- callers negate.
template <class F>
HD void mul_by_xabs(jac<F> &r, const jac<F> &p) {
  jac<F> acc = p;
  for (int i = 62; i >= 0; i--) {
    jac_dbl(acc, acc);
    if ((k::X_ABS >> i) & 1) jac_add(acc, acc, p);
  }
  r = acc;
}

// ----- on-curve checks
HD bool g1_on_curve(const g1a &a) {
  fp l, rr;
  fp_sqr(l, a.y);
  fp_sqr(rr, a.x);
  fp_mul(rr, rr, a.x);
  fp_add(rr, rr, fp_const(k::B1_M));
  return fp_eq(l, rr);
}
HD bool g2_on_curve(const g2a &a) {
  fp2 l, rr;
  fp2_sqr(l, a.y);
  fp2_sqr(rr, a.x);
  fp2_mul(rr, rr, a.x);
  fp2_add(rr, rr, fp2_const(k::B2_C0, k::B2_C1));
  return fp2_eq(l, rr);
}

// ----- endomorphisms
// psi(x,y) = (conj(x) cx, conj(y) cy); on Jacobian coordinates Z is conjugated too.
HD void g2_psi(g2j &r, const g2j &p) {
  fp2 t;
  fp2_conj(t, p.x);
  fp2_mul(r.x, t, fp2_const(k::PSI_CX_C0, k::PSI_CX_C1));
  fp2_conj(t, p.y);
  fp2_mul(r.y, t, fp2_const(k::PSI_CY_C0, k::PSI_CY_C1));
  fp2_conj(r.z, p.z);
}
HD void g2_psi2(g2j &r, const g2j &p) {
  fp2_mul(r.x, p.x, fp2_const(k::PSI2_CX_C0, k::PSI2_CX_C1));
  fp2_mul(r.y, p.y, fp2_const(k::PSI2_CY_C0, k::PSI2_CY_C1));
  r.z = p.z;
}

// G2 membership (affine input, assumed on curve): psi(P) == [x]P  (x < 0)
HD bool g2_in_group(const g2a &a) {
  if (aff_is_inf(a)) return true;
  g2j p, xp, pp;
  jac_from_aff(p, a);
  mul_by_xabs(xp, p);
  jac_neg(xp, xp);
  g2_psi(pp, p);
  return jac_eq(pp, xp);
}
// G1 membership: phi(P) = (beta x, y) == [-x^2]P
HD bool g1_in_group(const g1a &a) {
  if (aff_is_inf(a)) return true;
  g1j p, t;
  jac_from_aff(p, a);
  mul_by_xabs(t, p);
  mul_by_xabs(t, t);
  jac_neg(t, t);
  g1j phi;
  fp_mul(phi.x, a.x, fp_const(k::BETA_M));
  phi.y = a.y;
  fp_one(phi.z);
  return jac_eq(phi, t);
}

// ----- serialization (ZCash / blst big-endian compressed form)
HD void fp_from_be48(fp &r, const uint8_t *b) {
#pragma unroll
  for (int i = 0; i < 12; i++) {
    const uint8_t *q = b + 4 * (11 - i);
    r.l[i] = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | q[3];
  }
}
HD void fp_to_be48(uint8_t *b, const fp &a) {
#pragma unroll
  for (int i = 0; i < 12; i++) {
    uint8_t *q = b + 4 * (11 - i);
    uint32_t v = a.l[i];
    q[0] = v >> 24;
    q[1] = v >> 16;
    q[2] = v >> 8;
    q[3] = v;
  }
}

enum : int32_t {
  ST_SUCCESS = 0,
  ST_BAD_ENCODING = 1,
  ST_NOT_ON_CURVE = 2,
  ST_NOT_IN_GROUP = 3,
  ST_AGGR_TYPE_MISMATCH = 4,
  ST_VERIFY_FAIL = 5,
  ST_PK_IS_INFINITY = 6,
  ST_BAD_SCALAR = 7,
};

// blst POINTonE1_Uncompress_Z semantics
HD int32_t g1_decompress(g1a &r, const uint8_t *in) {
  f_zero(r.x);
  f_zero(r.y);
  uint8_t b0 = in[0];
  if (!(b0 & 0x80)) return ST_BAD_ENCODING;
  if (b0 & 0x40) {
    uint32_t acc = b0 & 0x3f;
    for (int i = 1; i < 48; i++) acc |= in[i];
    return acc ? ST_BAD_ENCODING : ST_SUCCESS;
  }
  fp x;
  fp_from_be48(x, in);
  x.l[11] &= 0x1fffffffu;
  if (!limbs_lt(x.l, k::P)) return ST_BAD_ENCODING;
  fp_to_mont(x, x);
  fp rhs, y;
  fp_sqr(rhs, x);
  fp_mul(rhs, rhs, x);
  fp_add(rhs, rhs, fp_const(k::B1_M));
  if (!fp_sqrt(y, rhs)) return ST_NOT_ON_CURVE;
  if (fp_lex_largest(y) != (bool)(b0 & 0x20)) fp_neg(y, y);
  r.x = x;
  r.y = y;
  if (fp_is_zero(x)) return ST_NOT_IN_GROUP;  // (0, +-2) has order 3
  return ST_SUCCESS;
}
// fp2_sqrt (bls_field.h) with the (p-3)/4 exponentiation as a policy, so that the latency
// regime can run its two exponentiations row-distributed (bls_dfp.h, k_g2_decompress_row)
template <class Pow>
HD bool fp2_sqrt_pow(fp2 &r, const fp2 &a, const Pow &pow) {
  if (fp2_is_zero(a)) {
    fp2_zero(r);
    return true;
  }
  fp n, t, gamma, g2;
  fp_sqr(n, a.c0);
  fp_sqr(t, a.c1);
  fp_add(n, n, t);
  pow(gamma, n);
  fp_mul(gamma, gamma, n);  // n^((p+1)/4)
  fp_sqr(g2, gamma);
  if (!fp_eq(g2, n)) return false;
  fp delta, x0, x0sq, tmp;
  fp_add(delta, a.c0, gamma);
  fp_half(delta, delta);
  if (fp_is_zero(delta)) {  // only when a1 == 0 and gamma == -a0
    fp_sub(delta, a.c0, gamma);
    fp_half(delta, delta);
  }
  pow(t, delta);
  fp_mul(x0, delta, t);
  fp_sqr(x0sq, x0);
  fp half_a1t;
  fp_mul(tmp, a.c1, t);
  fp_half(half_a1t, tmp);
  const bool sq = fp_eq(x0sq, delta);
  fp nh;
  fp_neg(nh, half_a1t);
  fp_sel(r.c0, sq, nh, x0);
  fp_sel(r.c1, sq, x0, half_a1t);
  fp2 chk;
  fp2_sqr(chk, r);
  return fp2_eq(chk, a);
}
struct LanePowCurve {
  HD void operator()(fp &r, const fp &a) const { fp_pow_pm3d4(r, a); }
};

// blst POINTonE2_Uncompress_Z semantics (on-curve check only)
template <class Pow>
HD int32_t g2_decompress_pow(g2a &r, const uint8_t *in, const Pow &pow) {
  f_zero(r.x);
  f_zero(r.y);
  uint8_t b0 = in[0];
  if (!(b0 & 0x80)) return ST_BAD_ENCODING;
  if (b0 & 0x40) {
    uint32_t acc = b0 & 0x3f;
    for (int i = 1; i < 96; i++) acc |= in[i];
    return acc ? ST_BAD_ENCODING : ST_SUCCESS;
  }
  fp2 x;
  fp_from_be48(x.c1, in);
  x.c1.l[11] &= 0x1fffffffu;
  fp_from_be48(x.c0, in + 48);
  if (!limbs_lt(x.c1.l, k::P) || !limbs_lt(x.c0.l, k::P)) return ST_BAD_ENCODING;
  fp_to_mont(x.c0, x.c0);
  fp_to_mont(x.c1, x.c1);
  fp2 rhs, y;
  fp2_sqr(rhs, x);
  fp2_mul(rhs, rhs, x);
  fp2_add(rhs, rhs, fp2_const(k::B2_C0, k::B2_C1));
  if (!fp2_sqrt_pow(y, rhs, pow)) return ST_NOT_ON_CURVE;
  if (fp2_lex_largest(y) != (bool)(b0 & 0x20)) fp2_neg(y, y);
  r.x = x;
  r.y = y;
  return ST_SUCCESS;
}
HD int32_t g2_decompress(g2a &r, const uint8_t *in) { return g2_decompress_pow(r, in, LanePowCurve()); }
HD void g1_compress(uint8_t *out, const g1a &a) {
  if (aff_is_inf(a)) {
    out[0] = 0xc0;
    for (int i = 1; i < 48; i++) out[i] = 0;
    return;
  }
  fp x;
  fp_from_mont(x, a.x);
  fp_to_be48(out, x);
  out[0] |= 0x80 | (fp_lex_largest(a.y) ? 0x20 : 0);
}
HD void g2_compress(uint8_t *out, const g2a &a) {
  if (aff_is_inf(a)) {
    out[0] = 0xc0;
    for (int i = 1; i < 96; i++) out[i] = 0;
    return;
  }
  fp x0, x1;
  fp_from_mont(x1, a.x.c1);
  fp_from_mont(x0, a.x.c0);
  fp_to_be48(out, x1);
  fp_to_be48(out + 48, x0);
  out[0] |= 0x80 | (fp2_lex_largest(a.y) ? 0x20 : 0);
}

}  // namespace gbls
