// G2 in the radix-2^28 field layer (bls_field28.h) for the lane-regime cofactor clearing
// (DESIGN.md section 8's migration order): the engine's Jacobian formulas
// (bls_curve.h jac_dbl / jac_add / mul_by_xabs, templates over the coordinate field) are
// instantiated for r28::fe2 through the overload set below, found by argument-dependent lookup.
// Every f_ operation returns a normalized, weakly reduced value (< 1.03 p), so each formula's
// inputs meet fe2_mul / fe2_sqr's bounds without bookkeeping; the doubling (jac_dbl28) and the
// Miller doubling step (line_dbl28), which dominate the chains, are written with lazy
// combinations and their bounds instead.  A product costs ~0.84 us per lane instead of the
// engine's ~1.18 (tools/ubench/r28_bench.hip).
#pragma once
#include "bls_curve.h"
#include "bls_pairing.h"
#include "bls_field28.h"
#include "bls_r28_consts.h"

namespace gbls {
namespace r28 {

HD void f_add(fe2 &r, const fe2 &a, const fe2 &b) { fe2_add_r(r, a, b); }
HD void f_sub(fe2 &r, const fe2 &a, const fe2 &b) { fe2_sub_r(r, a, b); }
HD void f_mul(fe2 &r, const fe2 &a, const fe2 &b) { fe2_mul(r, a, b); }
HD void f_sqr(fe2 &r, const fe2 &a) { fe2_sqr(r, a); }
HD void f_dbl(fe2 &r, const fe2 &a) { fe2_add_r(r, a, a); }
HD void f_zero(fe2 &r) {
#pragma unroll
  for (int i = 0; i < 14; i++) r.c0.l[i] = r.c1.l[i] = 0;
}
HD void f_neg(fe2 &r, const fe2 &a) {
  fe2 z;
  f_zero(z);
  fe2_sub_r(r, z, a);
}
HD void f_one(fe2 &r) {
  r.c0 = K28_ONE;
#pragma unroll
  for (int i = 0; i < 14; i++) r.c1.l[i] = 0;
}
HD bool f_is_zero(const fe2 &a) { return is_zero(a.c0) && is_zero(a.c1); }
HD bool f_eq(const fe2 &a, const fe2 &b) {  // a, b normalized, < 4 p
  fe2 d;
  fe2_sub(d, a, b);
  return f_is_zero(d);
}

// the lazy combinations (bls_field28.h) jac_dbl28 is written in
HD void f_add_n(fe2 &r, const fe2 &a, const fe2 &b) { fe2_add_n(r, a, b); }
HD void f_sub_n(fe2 &r, const fe2 &a, const fe2 &b) { fe2_sub(r, a, b); }
HD void f_mulk_n(fe2 &r, const fe2 &a, uint32_t k) { fe2_mulk_n(r, a, k); }
template <uint32_t K>
HD void f_subk_r(fe2 &r, const fe2 &a, const fe2 &b) {
  fe2_subk_r<K>(r, a, b);
}
template <uint32_t S>
HD void f_sub2_r(fe2 &r, const fe2 &a, const fe2 &b, const fe2 &c) {
  fe2_sub2_r<S>(r, a, b, c);
}
template <uint32_t S, uint32_t K>
HD void f_lin_r(fe2 &r, const fe2 &a, const fe2 &b) {
  fe2_lin_r<S, K>(r, a, b);
}
template <uint32_t S, uint32_t K1, uint32_t K2>
HD void f_lin_r(fe2 &r, const fe2 &a, const fe2 &b, const fe2 &c) {
  fe2_lin_r<S, K1, K2>(r, a, b, c);
}

typedef jac<fe2> g2j28;

// dbl-2009-l as bls_curve.h jac_dbl, with lazy combinations: one normalization per combination
// and a weak reduction only for D, X3 and Y3 (3 per coordinate field element, against 14 when
// every addition reduces).  The jac_dbl overloads for g2j28 / g1j28 below take precedence over
// bls_curve.h's template (argument-dependent lookup finds them from every caller, including
// mul_by_xabs and jac_add's degenerate case).
// Contract: input coordinates normalized and < 2.1 p; X3, Y3 < 1.03 p, Z3 normalized and
// < 2.03 p, which every point routine of this layer accepts (jac_add's products and f_add,
// f_neg of Y, psi, the conversions, is_zero).  r may alias p.
template <class F>
HD void jac_dbl28(jac<F> &r, const jac<F> &p) {
  F A, B, C, t;
  f_mul(t, p.y, p.z);
  f_sqr(A, p.x);
  f_sqr(B, p.y);
  f_add_n(C, p.x, B);       // X + B (< 3.2 p)
  f_add_n(r.z, t, t);       // Z3 = 2YZ (< 2.03 p)   (p.y, p.z dead)
  f_sqr(t, C);              // (X + B)^2             (p.x dead)
  f_sqr(C, B);              // C = B^2               (B dead)
  f_sub2_r<2>(B, t, A, C);  // D = 2((X+B)^2 - A - C)
  f_mulk_n(A, A, 3);        // E = 3A (< 3.1 p)
  f_sqr(t, A);              // F = E^2
  f_subk_r<2>(r.x, t, B);   // X3 = F - 2D
  f_sub_n(t, B, r.x);       // D - X3 (< 5.1 p)
  f_mul(t, A, t);           // E (D - X3)
  f_subk_r<8>(r.y, t, C);   // Y3 = E (D - X3) - 8C
}
HD void jac_dbl(g2j28 &r, const g2j28 &p) { jac_dbl28(r, p); }

// add-2007-bl as bls_curve.h jac_add, with lazy combinations (3 weak reductions per field
// element fewer).  Contract as jac_dbl28: inputs normalized, < 2.1 p; outputs < 1.03 p.
// r may alias a (NOT b).
template <class F>
HD void jac_add28(jac<F> &r, const jac<F> &a, const jac<F> &b) {
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
  f_sub2_r<1>(t, t, z1z1, z2z2);  // 2 Z1 Z2             (z1z1, z2z2, a.* dead)
  f_sub(u2, u2, u1);              // H
  f_lin_r<2, 1>(s2, s2, s1);      // r = 2 (S2 - S1)
  if (f_is_zero(u2)) {
    if (f_is_zero(s2))
      jac_dbl(r, b);
    else
      jac_set_inf(r);
    return;
  }
  f_mul(r.z, t, u2);              // Z3 = 2 Z1 Z2 H
  f_add_n(t, u2, u2);
  f_sqr(t, t);                    // I = (2H)^2
  f_mul(u2, u2, t);               // J = H I
  f_mul(u1, u1, t);               // V = U1 I
  f_sqr(t, s2);
  f_lin_r<1, 1, 2>(r.x, t, u2, u1);  // X3 = r^2 - J - 2V
  f_sub_n(t, u1, r.x);            // V - X3 (< 5.1 p)
  f_mul(t, s2, t);
  f_mul(s1, s1, u2);
  f_lin_r<1, 2>(r.y, t, s1);      // Y3 = r (V - X3) - 2 S1 J
}

// madd-2007-bl as bls_curve.h jac_add_aff, lazy; CHECK_B = false when b is known finite (the
// MSM's bucket points: no zero test of b).  r may alias a.
template <bool CHECK_B, class F>
HD void jac_add_aff28(jac<F> &r, const jac<F> &a, const aff<F> &b) {
  if (CHECK_B && aff_is_inf(b)) {
    r = a;
    return;
  }
  if (jac_is_inf(a)) {
    r.x = b.x;
    r.y = b.y;
    f_one(r.z);
    if (CHECK_B && aff_is_inf(b)) f_zero(r.z);
    return;
  }
  F z1z1, u2, s2, t, hh;
  f_sqr(z1z1, a.z);
  f_mul(u2, b.x, z1z1);
  f_mul(s2, b.y, a.z);
  f_mul(s2, s2, z1z1);
  f_sub(u2, u2, a.x);             // H
  f_lin_r<2, 1>(s2, s2, a.y);     // r = 2 (S2 - Y1)
  if (f_is_zero(u2)) {
    if (f_is_zero(s2)) {
      jac<F> bj;
      bj.x = b.x;
      bj.y = b.y;
      f_one(bj.z);
      jac_dbl(r, bj);
    } else {
      jac_set_inf(r);
    }
    return;
  }
  f_add_n(t, a.z, u2);            // Z1 + H (< 3.2 p)
  f_sqr(t, t);
  f_sqr(hh, u2);
  f_sub2_r<1>(r.z, t, z1z1, hh);  // Z3 = (Z1 + H)^2 - Z1Z1 - HH   (a.z dead)
  f_mulk_n(hh, hh, 4);            // I = 4 HH (< 4.1 p)
  f_mul(z1z1, a.x, hh);           // V = X1 I
  f_mul(hh, u2, hh);              // J = H I
  f_mul(t, a.y, hh);              // Y1 J                    (a.x, a.y dead)
  f_sqr(u2, s2);
  f_lin_r<1, 1, 2>(r.x, u2, hh, z1z1);  // X3 = r^2 - J - 2V
  f_sub_n(u2, z1z1, r.x);         // V - X3 (< 5.1 p)
  f_mul(u2, s2, u2);
  f_lin_r<1, 2>(r.y, u2, t);      // Y3 = r (V - X3) - 2 Y1 J
}
typedef aff<fe2> g2a28;
HD void jac_add(g2j28 &r, const g2j28 &a, const g2j28 &b) { jac_add28(r, a, b); }
HD void jac_add_aff(g2j28 &r, const g2j28 &a, const g2a28 &b) { jac_add_aff28<true>(r, a, b); }

HD void g2j_in(g2j28 &r, const g2j &a) {
  from_fp(r.x.c0, a.x.c0);
  from_fp(r.x.c1, a.x.c1);
  from_fp(r.y.c0, a.y.c0);
  from_fp(r.y.c1, a.y.c1);
  from_fp(r.z.c0, a.z.c0);
  from_fp(r.z.c1, a.z.c1);
}
HD void g2j_out(g2j &r, const g2j28 &a) {
  to_fp(r.x.c0, a.x.c0);
  to_fp(r.x.c1, a.x.c1);
  to_fp(r.y.c0, a.y.c0);
  to_fp(r.y.c1, a.y.c1);
  to_fp(r.z.c0, a.z.c0);
  to_fp(r.z.c1, a.z.c1);
}
// psi(x, y, z) = (conj(x) cx, conj(y) cy, conj(z)) with cx = K28_PSI_CX1 u
HD void g2_psi28(g2j28 &r, const g2j28 &p) {
  fe2 t, c;
  t.c0 = p.x.c0;
  f_zero(c);
  sub_r(t.c1, c.c0, p.x.c1);  // conj(x)
  // (t0 + t1 u)(k u) = -t1 k + t0 k u
  fe n1;
  mul(n1, t.c1, K28_PSI_CX1);
  mul(r.x.c1, t.c0, K28_PSI_CX1);
  sub_r(r.x.c0, c.c0, n1);
  t.c0 = p.y.c0;
  sub_r(t.c1, c.c0, p.y.c1);  // conj(y)
  c.c0 = K28_PSI_CY0;
  c.c1 = K28_PSI_CY1;
  fe2_mul(r.y, t, c);
  r.z.c0 = p.z.c0;
  f_zero(c);
  sub_r(r.z.c1, c.c0, p.z.c1);
}
HD void g2_psi2_28(g2j28 &r, const g2j28 &p) {
  fe2_mul_fe(r.x, p.x, K28_PSI2_CX);
  fe2_mul_fe(r.y, p.y, K28_PSI2_CY);
  r.z = p.z;
}

// a / 2 mod p (a normalized, < 1.03 p): (a + (a odd ? p : 0)) / 2, normalized, < 1.02 p
HD void half(fe &r, const fe &a) {
  constexpr uint32_t P[14] = {GBLS_R28_P};
  const uint32_t odd = a.l[0] & 1u;
  fe s;
#pragma unroll
  for (int i = 0; i < 14; i++) s.l[i] = a.l[i] + (odd ? P[i] : 0u);
  norm(s);
#pragma unroll
  for (int i = 0; i < 13; i++) r.l[i] = (s.l[i] >> 1) | ((s.l[i + 1] & 1u) << 27);
  r.l[13] = s.l[13] >> 1;
}
HD void fe2_half(fe2 &r, const fe2 &a) {
  half(r.c0, a.c0);
  half(r.c1, a.c1);
}
// 3 b' a = 12 (1 + u) a = 12 (a0 - a1) + 12 (a0 + a1) u, weakly reduced (a normalized, < 4 p)
HD void fe2_mul_3b(fe2 &r, const fe2 &a) {
  fe s0, s1;
  sub(s0, a.c0, a.c1);  // < 5.1 p
  add_n(s1, a.c0, a.c1);
  mulk_r(r.c0, s0, 12);
  mulk_r(r.c1, s1, 12);
}

// ---------------------------------------------------------------- Miller line steps (k_lines)
// The lane regime's line steps (k_lines.hip lane_line_dbl / lane_line_add_aff, i.e.
// bls_pairing.h line_dbl / line_add_aff reordered so each coefficient is handed to `put` as soon
// as it is known) on a homogeneous point T over r28::fe2: the same operations on the same
// operands, so the same field values.  put(c, v) receives L0 (c = 0), L2 (c = 2), L3 (c = 4).
struct g2h28 {
  fe2 x, y, z;
};
// The additions are lazy (bls_field28.h "lazy point arithmetic"): each combination is
// normalized once and weakly reduced only where a coefficient is handed out or T is updated,
// so T keeps its bound (coordinates normalized, < 1.03 p) and every coefficient is < 1.03 p.
template <class Put>
HD void line_dbl28(g2h28 &T, Put &&put) {
  fe2 A, B, E, H, t;
  fe2_sqr(B, T.y);             // Y^2
  fe2_sqr(t, T.z);             // C = Z^2
  fe2_mul_3b(E, t);            // 3b'Z^2
  fe2_add_n(H, T.y, T.z);      // Y + Z (< 2.1 p)
  fe2_sqr(H, H);
  fe2_sub2_r<1>(H, H, B, t);   // 2YZ                      (C dead)
  fe2_mul(A, T.x, T.y);
  fe2_half(A, A);              // XY/2                     (Y dead)
  f_neg(t, H);
  put(4, t);                   // L3 = -2YZ
  fe2_sub_r(t, E, B);
  put(0, t);                   // L0 = 3b'Z^2 - Y^2
  fe2_sqr(t, T.x);
  fe2_mulk_r(t, t, 3);
  put(2, t);                   // L2 = 3X^2                (X dead)
  fe2 F;
  fe2_mulk_n(F, E, 3);         // 3E (< 3.1 p)
  fe2_sub(t, B, F);            // B - F (< 5.1 p)
  fe2_mul(T.x, A, t);          // X3 = A (B - F)
  fe2_mul(T.z, B, H);          // Z3 = B H
  fe2_add_n(t, B, F);
  fe2_half(t, t);              // G = (B + F) / 2 (< 2.6 p)
  fe2_sqr(t, t);               // G^2
  fe2_sqr(E, E);
  fe2_subk_r<3>(T.y, t, E);    // Y3 = G^2 - 3E^2
}
// T + Q for an affine Q = (qx, qy): theta = Y1 - y2 Z1, lambda = X1 - x2 Z1
template <class Put>
HD void line_add28(g2h28 &T, const fe2 &qx, const fe2 &qy, Put &&put) {
  fe2 th, la, t, u;
  fe2_mul(t, qy, T.z);
  fe2_sub_r(th, T.y, t);
  fe2_mul(t, qx, T.z);
  fe2_sub_r(la, T.x, t);
  fe2_mul(u, th, qx);
  fe2_mul(t, la, qy);
  fe2_sub_r(u, u, t);
  put(0, u);             // L0 = theta x2 - lambda y2
  f_neg(u, th);
  put(2, u);             // L2 = -theta
  put(4, la);            // L3 = lambda
  fe2 vv, vvv, R, A;
  fe2_sqr(u, th);        // uu
  fe2_sqr(vv, la);
  fe2_mul(vvv, vv, la);
  f_neg(vvv, vvv);       // v^3 = -lambda^3
  fe2_mul(R, vv, T.x);
  fe2_mul(A, u, T.z);
  fe2_sub_r(A, A, vvv);
  fe2_sub_r(A, A, R);
  fe2_sub_r(A, A, R);
  fe2_mul(T.x, la, A);
  f_neg(T.x, T.x);       // X3 = v A
  fe2_sub_r(t, R, A);
  fe2_mul(t, th, t);
  f_neg(t, t);           // u (R - A)
  fe2_mul(R, vvv, T.y);
  fe2_sub_r(T.y, t, R);
  fe2_mul(T.z, vvv, T.z);
}

// a radix-2^28 value stored in an engine-layout slot without conversion: the 392-bit limb
// vector of a normalized value < 2^384 repacked into 12 words (no product: the value times
// 2^392 mod p, which an engine-form reader sees as the value times 2^8)
HD void store12(fp &dst, const fe &a) { repack_out(dst, a); }
HD void load12(fe &r, const fp &src) { repack_in(r, src); }
// points in engine-layout slots, coordinate by coordinate (store12 / load12): the clearing
// chains' intermediate points and the MSM's signatures and bucket partials
HD void g2j_store12(g2j &dst, const g2j28 &a) {
  store12(dst.x.c0, a.x.c0), store12(dst.x.c1, a.x.c1);
  store12(dst.y.c0, a.y.c0), store12(dst.y.c1, a.y.c1);
  store12(dst.z.c0, a.z.c0), store12(dst.z.c1, a.z.c1);
}
HD void g2j_load12(g2j28 &r, const g2j &src) {
  load12(r.x.c0, src.x.c0), load12(r.x.c1, src.x.c1);
  load12(r.y.c0, src.y.c0), load12(r.y.c1, src.y.c1);
  load12(r.z.c0, src.z.c0), load12(r.z.c1, src.z.c1);
}
HD void g2a_store12(g2a &dst, const g2a28 &a) {
  store12(dst.x.c0, a.x.c0), store12(dst.x.c1, a.x.c1);
  store12(dst.y.c0, a.y.c0), store12(dst.y.c1, a.y.c1);
}
HD void g2a_load12(g2a28 &r, const g2a &src) {
  load12(r.x.c0, src.x.c0), load12(r.x.c1, src.x.c1);
  load12(r.y.c0, src.y.c0), load12(r.y.c1, src.y.c1);
}

// 1/a (0 -> 0) through the engine's safegcd inversion (bls_field.h fp_inv): a < 16 p
HD void inv(fe &r, const fe &a) {
  fp t;
  to_fp(t, a);
  fp_inv(t, t);
  from_fp(r, t);
}
// 1/a = conj(a) / N(a) (0 -> 0): a normalized, < 2.1 p
HD void fe2_inv(fe2 &r, const fe2 &a) {
  fe n, t;
  sqr(n, a.c0);
  sqr(t, a.c1);
  add_n(n, n, t);
  inv(n, n);
  mul(r.c0, a.c0, n);
  mul(t, a.c1, n);
  fe z;
#pragma unroll
  for (int i = 0; i < 14; i++) z.l[i] = 0;
  sub_r(r.c1, z, t);
}
// Jacobian -> affine, infinity -> (0, 0)
HD void jac_to_aff28(g2a28 &r, const g2j28 &p) {
  fe2 zi, zi2, zi3;
  fe2_inv(zi, p.z);
  fe2_sqr(zi2, zi);
  fe2_mul(zi3, zi2, zi);
  fe2_mul(r.x, p.x, zi2);
  fe2_mul(r.y, p.y, zi3);
}
// [|x|] b for an affine base ((0, 0): infinity, whose chain runs on garbage and is dropped): 63
// lazy doublings and 5 mixed additions -- 256 VGPRs, no scratch, so two waves per SIMD
// (tools/ubench/occ28_bench.hip).  b may live in LDS.
HD void g2_xabs_aff28(g2j28 &r, const g2a28 &b) {
  g2j28 acc;
  acc.x = b.x;
  acc.y = b.y;
  f_one(acc.z);
  for (int i = 62; i >= 0; i--) {
    jac_dbl(acc, acc);
    if ((k::X_ABS >> i) & 1) jac_add_aff28<false>(acc, acc, b);
  }
  if (f_is_zero(b.x) && f_is_zero(b.y)) jac_set_inf(acc);
  r = acc;
}
HD void g2j_of_aff28(g2j28 &r, const g2a28 &a) {
  r.x = a.x;
  r.y = a.y;
  f_one(r.z);
  if (f_is_zero(a.x) && f_is_zero(a.y)) jac_set_inf(r);
}

// G2 membership in radix 2^28 (bls_curve.h g2_in_group: psi(P) == [x]P, x < 0) for an affine
// point that is not infinity, in radix-2^28 form; the affine base may be parked in LDS by the
// caller (k_g2_check28)
HD bool g2_in_group28(const g2a28 &b) {
  g2j28 acc;
  g2_xabs_aff28(acc, b);
  jac_neg(acc, acc);  // [x]P
  g2j28 p, pp;
  g2j_of_aff28(p, b);
  g2_psi28(pp, p);
  return jac_eq(pp, acc);
}

// The lane-regime cofactor clearing in stages (k_h2c_clear.hip), with both [|x|] chains on
// affine bases (g2_xabs_aff28, their own two-waves-per-SIMD kernel):
//   pre:   P = Q0 + Q1, affine
//   chain: X1 = [|x|] P
//   mid:   t1 = -X1 = [x]P;  t2 = t1 + psi(P) (affine);  T = X1 - P + psi^2(2P) - psi(P)
//   chain: X2 = [|x|] t2
//   post:  h = T - X2 = [x^2 - x - 1]P + [x - 1]psi(P) + psi^2(2P)   (clear_cofactor_g2)
HD void clear_mid28(g2a28 &t2a, g2j28 &T, const g2a28 &pa, const g2j28 &x1) {
  g2j28 p, t1, t2, v;
  g2j_of_aff28(p, pa);
  jac_neg(t1, x1);  // [x]P
  g2_psi28(t2, p);
  jac_add(t2, t2, t1);  // t1 + psi(P)
  jac_to_aff28(t2a, t2);
  jac_neg(v, p);
  jac_add(T, x1, v);  // - t1 - P
  jac_dbl(v, p);
  g2_psi2_28(v, v);
  jac_add(T, T, v);  // + psi^2(2P)
  g2_psi28(v, p);
  jac_neg(v, v);
  jac_add(T, T, v);  // - psi(P)
}
HD void clear_post28(g2j28 &h, const g2j28 &x2, const g2j28 &T) {
  jac_neg(h, x2);
  jac_add(h, h, T);
}
// the stages in sequence (host tests)
HD void clear_cofactor28_staged(g2j28 &r, const g2j28 &p) {
  g2a28 pa, t2a;
  g2j28 x1, x2, T;
  jac_to_aff28(pa, p);
  g2_xabs_aff28(x1, pa);
  clear_mid28(t2a, T, pa, x1);
  g2_xabs_aff28(x2, t2a);
  clear_post28(r, x2, T);
}

// h_eff P, the sequence of clear_cofactor_g2 (bls_hash.h, Budroni-Pintore): host tests of
// the layer's G2 formulas (tests/native/host_harness.cpp)
HD void clear_cofactor28(g2j28 &r, const g2j28 &p) {
  g2j28 t1, t2, t3;
  mul_by_xabs(t1, p);
  jac_neg(t1, t1);  // t1 = [x]P
  g2_psi28(t2, p);
  jac_add(t2, t2, t1);  // t1 + psi(P)
  mul_by_xabs(t3, t2);
  jac_neg(t3, t3);  // t3 = [x](t1 + psi(P))
  jac_neg(t1, t1);
  jac_add(t3, t3, t1);  // - t1
  jac_dbl(t1, p);
  g2_psi2_28(t1, t1);
  jac_add(t3, t3, t1);  // + psi^2(2P)
  g2_psi28(t1, p);
  jac_neg(t1, t1);
  jac_add(t3, t3, t1);  // - psi(P)
  jac_neg(t1, p);
  jac_add(r, t3, t1);  // - P
}

// ---------------------------------------------------------------- G1 (k_mv_g1mul_lane28)
// The same Jacobian templates over r28::fe (weakly reduced values < 1.03 p, as for fe2);
// squarings take the dedicated radix-2^28 square (sqr: 105 + 196 product terms).
HD void f_add(fe &r, const fe &a, const fe &b) {
  add(r, a, b);
  wred(r);
}
HD void f_sub(fe &r, const fe &a, const fe &b) { sub_r(r, a, b); }
HD void f_mul(fe &r, const fe &a, const fe &b) { mul(r, a, b); }
HD void f_sqr(fe &r, const fe &a) { sqr(r, a); }
HD void f_dbl(fe &r, const fe &a) { f_add(r, a, a); }
HD void f_zero(fe &r) {
#pragma unroll
  for (int i = 0; i < 14; i++) r.l[i] = 0;
}
HD void f_neg(fe &r, const fe &a) {
  fe z;
  f_zero(z);
  sub_r(r, z, a);
}
HD void f_one(fe &r) { r = K28_ONE; }
HD bool f_is_zero(const fe &a) { return is_zero(a); }
HD bool f_eq(const fe &a, const fe &b) {
  fe d;
  sub(d, a, b);
  return is_zero(d);
}

HD void f_add_n(fe &r, const fe &a, const fe &b) { add_n(r, a, b); }
HD void f_sub_n(fe &r, const fe &a, const fe &b) { sub(r, a, b); }
HD void f_mulk_n(fe &r, const fe &a, uint32_t k) { mulk_n(r, a, k); }
template <uint32_t K>
HD void f_subk_r(fe &r, const fe &a, const fe &b) {
  subk_r<K>(r, a, b);
}
template <uint32_t S>
HD void f_sub2_r(fe &r, const fe &a, const fe &b, const fe &c) {
  sub2_r<S>(r, a, b, c);
}
template <uint32_t S, uint32_t K>
HD void f_lin_r(fe &r, const fe &a, const fe &b) {
  lin_r<S, K>(r, a, b);
}
template <uint32_t S, uint32_t K1, uint32_t K2>
HD void f_lin_r(fe &r, const fe &a, const fe &b, const fe &c) {
  lin_r<S, K1, K2>(r, a, b, c);
}

typedef jac<fe> g1j28;
HD void jac_dbl(g1j28 &r, const g1j28 &p) { jac_dbl28(r, p); }
HD void jac_add(g1j28 &r, const g1j28 &a, const g1j28 &b) { jac_add28(r, a, b); }

HD void g1j28_sel(g1j28 &r, bool c, const g1j28 &a, const g1j28 &b) {  // c ? b : a
#pragma unroll
  for (int i = 0; i < 14; i++) {
    r.x.l[i] = c ? b.x.l[i] : a.x.l[i];
    r.y.l[i] = c ? b.y.l[i] : a.y.l[i];
    r.z.l[i] = c ? b.z.l[i] : a.z.l[i];
  }
}
// [k] base for a 64-bit k: g1_mul_u64_w3 (bls_curve.h: signed 3-bit windows, the same
// instructions for every lane's scalar) over r28::fe; base affine, engine form
HD void g1_mul_u64_w3_28(g1j28 &r, const g1a &base, uint64_t k) {
  g1j28 t0, t1, t2, t3;
  from_fp(t0.x, base.x);
  from_fp(t0.y, base.y);
  f_one(t0.z);
  if (aff_is_inf(base)) f_zero(t0.z);  // (0, 0): the point at infinity
  jac_dbl(t1, t0);
  jac_add(t2, t1, t0);
  jac_dbl(t3, t1);
  uint32_t cmask = 0, carry = 0;
#pragma unroll
  for (int i = 0; i < 22; i++) {
    cmask |= carry << i;
    carry = ((uint32_t)((k >> (3 * i)) & 7u) + carry) > 4;  // 3 i <= 63
  }
  g1j28 acc;
  jac_set_inf(acc);
  const uint32_t top = (uint32_t)(k >> 63) + (cmask >> 21);  // top digit in [0, 2]
  g1j28_sel(acc, top == 1, acc, t0);
  g1j28_sel(acc, top == 2, acc, t1);
#pragma unroll 1
  for (int i = 20; i >= 0; i--) {
    jac_dbl(acc, acc);
    jac_dbl(acc, acc);
    jac_dbl(acc, acc);
    int v = (int)((k >> (3 * i)) & 7u) + (int)((cmask >> i) & 1u);
    if (v > 4) v -= 8;
    const uint32_t m = (uint32_t)(v < 0 ? -v : v);
    g1j28 q = t0, sum;
    g1j28_sel(q, m == 2, q, t1);
    g1j28_sel(q, m == 3, q, t2);
    g1j28_sel(q, m == 4, q, t3);
    fe ny;
    f_neg(ny, q.y);
    if (v < 0) q.y = ny;
    jac_add(sum, acc, q);
    g1j28_sel(acc, m != 0, acc, sum);
  }
  r = acc;
}
// g1s_from_jac (bls_pairing.h) of a radix-2^28 point: (X Z, Y, Z^3) in engine form
HD void g1s_from_jac28(g1s &r, const g1j28 &p) {
  if (jac_is_inf(p)) {
    fp_zero(r.x);
    fp_zero(r.y);
    fp_zero(r.c);
    return;
  }
  fe z2, t;
  sqr(z2, p.z);
  mul(t, z2, p.z);
  to_fp(r.c, t);
  mul(t, p.x, p.z);
  to_fp(r.x, t);
  to_fp(r.y, p.y);
}

}  // namespace r28
}  // namespace gbls
