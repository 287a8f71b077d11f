// BLS12-381 field tower for gfx950: Fp (12 x 32-bit limbs, Montgomery R = 2^384),
// Fp2 = Fp[u]/(u^2+1), Fp6 = Fp2[v]/(v^3-(1+u)), Fp12 = Fp6[w]/(w^2-v).
//
// Replaces blst 0.3.11's fp/fp2/fp12 layer (reached from bls/src/signature.rs:50-57,
// 85-90, 117-126 through the blst crate).  One lane owns one element; arithmetic is
// VALU integer work (v_mad_u64_u32 chains), never MFMA.  Every value is kept fully
// reduced (< p), so limb-wise equality is field equality.  Functions are
// __host__ __device__ so the host test harness (tests/native) can exercise the exact
// code the kernels run.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bls_constants.h"

#define HD __host__ __device__ __forceinline__
#define HDNI __host__ __device__ __noinline__

namespace gbls {

struct fp {
  uint32_t l[12];
};
struct fp2 {
  fp c0, c1;
};
struct fp6 {
  fp2 c0, c1, c2;
};
struct fp12 {
  fp6 c0, c1;
};

// ---------------------------------------------------------------- limb helpers
HD uint32_t addc(uint32_t a, uint32_t b, uint32_t &c) {
  uint64_t s = (uint64_t)a + b + c;
  c = (uint32_t)(s >> 32);
  return (uint32_t)s;
}
HD uint32_t subb(uint32_t a, uint32_t b, uint32_t &br) {
  uint64_t d = (uint64_t)a - b - br;
  br = (uint32_t)(d >> 63);
  return (uint32_t)d;
}

HD void fp_set(fp &r, const uint32_t (&c)[12]) {
#pragma unroll
  for (int i = 0; i < 12; i++) r.l[i] = c[i];
}
HD fp fp_const(const uint32_t (&c)[12]) {
  fp r;
  fp_set(r, c);
  return r;
}
HD void fp_zero(fp &r) {
#pragma unroll
  for (int i = 0; i < 12; i++) r.l[i] = 0;
}
HD void fp_one(fp &r) { fp_set(r, k::ONE_M); }
HD bool fp_is_zero(const fp &a) {
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) acc |= a.l[i];
  return acc == 0;
}
HD bool fp_eq(const fp &a, const fp &b) {
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) acc |= a.l[i] ^ b.l[i];
  return acc == 0;
}
HD bool fp_is_one(const fp &a) { return fp_eq(a, fp_const(k::ONE_M)); }
// r = c ? b : a   (branch-free select)
HD void fp_sel(fp &r, bool c, const fp &a, const fp &b) {
  uint32_t m = 0u - (uint32_t)c;
#pragma unroll
  for (int i = 0; i < 12; i++) r.l[i] = (a.l[i] & ~m) | (b.l[i] & m);
}
// a < b on canonical limbs
HD bool limbs_lt(const uint32_t *a, const uint32_t (&b)[12]) {
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) (void)subb(a[i], b[i], br);
  return br != 0;
}

// ---------------------------------------------------------------- Fp
HD void fp_add(fp &r, const fp &a, const fp &b) {
  uint32_t s[12], t[12], c = 0, br = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) s[i] = addc(a.l[i], b.l[i], c);
#pragma unroll
  for (int i = 0; i < 12; i++) t[i] = subb(s[i], k::P[i], br);
  uint32_t m = 0u - br;  // br=1 -> s < p -> keep s
#pragma unroll
  for (int i = 0; i < 12; i++) r.l[i] = (t[i] & ~m) | (s[i] & m);
}
HD void fp_sub(fp &r, const fp &a, const fp &b) {
  uint32_t d[12], br = 0, c = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) d[i] = subb(a.l[i], b.l[i], br);
  uint32_t m = 0u - br;
#pragma unroll
  for (int i = 0; i < 12; i++) r.l[i] = addc(d[i], k::P[i] & m, c);
}
HD void fp_dbl(fp &r, const fp &a) { fp_add(r, a, a); }
HD void fp_neg(fp &r, const fp &a) {
  fp z;
  fp_zero(z);
  fp_sub(r, z, a);
}

// Montgomery product, "no-carry" CIOS (valid because p[11] < 2^31 - 1):
// 2 x 144 v_mad_u64_u32 per product, result < 2p then one conditional subtract.
// The outer loop is kept rolled (b is rotated through registers) so that the many
// inlined call sites stay compact; the inner 12-limb row is fully unrolled.
HD void fp_mul(fp &r, const fp &a, const fp &b) {
  uint32_t t[12], bb[12];
#pragma unroll
  for (int j = 0; j < 12; j++) {
    t[j] = 0;
    bb[j] = b.l[j];
  }
#pragma unroll 1
  for (int i = 0; i < 12; i++) {
    const uint32_t bi = bb[0];
#pragma unroll
    for (int j = 0; j < 11; j++) bb[j] = bb[j + 1];
    uint64_t s = (uint64_t)a.l[0] * bi + t[0];
    uint32_t A = (uint32_t)(s >> 32);
    uint32_t t0 = (uint32_t)s;
    uint32_t m = t0 * k::PINV;
    uint64_t s2 = (uint64_t)m * k::P[0] + t0;
    uint32_t C = (uint32_t)(s2 >> 32);
#pragma unroll
    for (int j = 1; j < 12; j++) {
      s = (uint64_t)a.l[j] * bi + t[j] + A;
      A = (uint32_t)(s >> 32);
      s2 = (uint64_t)m * k::P[j] + (uint32_t)s + C;
      C = (uint32_t)(s2 >> 32);
      t[j - 1] = (uint32_t)s2;
    }
    t[11] = A + C;
  }
  uint32_t u[12], br = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) u[i] = subb(t[i], k::P[i], br);
  uint32_t msk = 0u - br;
#pragma unroll
  for (int i = 0; i < 12; i++) r.l[i] = (u[i] & ~msk) | (t[i] & msk);
}
HD void fp_sqr(fp &r, const fp &a) { fp_mul(r, a, a); }

HD void fp_to_mont(fp &r, const fp &a) { fp_mul(r, a, fp_const(k::R2)); }
HD void fp_from_mont(fp &r, const fp &a) {
  fp one;
  fp_zero(one);
  one.l[0] = 1;
  fp_mul(r, a, one);
}
HD void fp_mul3(fp &r, const fp &a) {
  fp t;
  fp_add(t, a, a);
  fp_add(r, t, a);
}

// a^e for a public constant exponent e (12 limbs); the branch is wave-uniform.
HDNI void fp_pow(fp &r, const fp &a, const uint32_t (&e)[12]) {
  fp acc;
  fp_one(acc);
  bool started = false;
  for (int i = 383; i >= 0; i--) {
    if (started) fp_sqr(acc, acc);
    if ((e[i >> 5] >> (i & 31)) & 1) {
      if (started)
        fp_mul(acc, acc, a);
      else
        acc = a;
      started = true;
    }
  }
  r = acc;
}
HD void fp_inv(fp &r, const fp &a) { fp_pow(r, a, k::EXP_PM2); }
// returns true iff a is a square; r = a^((p+1)/4) (a square root when it exists)
HD bool fp_sqrt(fp &r, const fp &a) {
  fp s, s2;
  fp_pow(s, a, k::EXP_SQRT);
  fp_sqr(s2, s);
  r = s;
  return fp_eq(s2, a);
}
// sort flag of the ZCash encoding: canonical(a) > (p-1)/2
HD bool fp_lex_largest(const fp &a) {
  fp c;
  fp_from_mont(c, a);
  // c > HALF_P  <=>  HALF_P < c
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) (void)subb(k::HALF_P[i], c.l[i], br);
  return br != 0;
}
HD uint32_t fp_parity(const fp &a) {
  fp c;
  fp_from_mont(c, a);
  return c.l[0] & 1;
}

// ---------------------------------------------------------------- Fp2
HD void fp2_zero(fp2 &r) {
  fp_zero(r.c0);
  fp_zero(r.c1);
}
HD void fp2_one(fp2 &r) {
  fp_one(r.c0);
  fp_zero(r.c1);
}
HD fp2 fp2_const(const uint32_t (&a)[12], const uint32_t (&b)[12]) {
  fp2 r;
  fp_set(r.c0, a);
  fp_set(r.c1, b);
  return r;
}
HD bool fp2_is_zero(const fp2 &a) { return fp_is_zero(a.c0) && fp_is_zero(a.c1); }
HD bool fp2_eq(const fp2 &a, const fp2 &b) { return fp_eq(a.c0, b.c0) && fp_eq(a.c1, b.c1); }
HD void fp2_sel(fp2 &r, bool c, const fp2 &a, const fp2 &b) {
  fp_sel(r.c0, c, a.c0, b.c0);
  fp_sel(r.c1, c, a.c1, b.c1);
}
HD void fp2_add(fp2 &r, const fp2 &a, const fp2 &b) {
  fp_add(r.c0, a.c0, b.c0);
  fp_add(r.c1, a.c1, b.c1);
}
HD void fp2_sub(fp2 &r, const fp2 &a, const fp2 &b) {
  fp_sub(r.c0, a.c0, b.c0);
  fp_sub(r.c1, a.c1, b.c1);
}
HD void fp2_dbl(fp2 &r, const fp2 &a) { fp2_add(r, a, a); }
HD void fp2_neg(fp2 &r, const fp2 &a) {
  fp_neg(r.c0, a.c0);
  fp_neg(r.c1, a.c1);
}
HD void fp2_conj(fp2 &r, const fp2 &a) {
  r.c0 = a.c0;
  fp_neg(r.c1, a.c1);
}
// Karatsuba: 3 Fp products
HD void fp2_mul(fp2 &r, const fp2 &a, const fp2 &b) {
  fp t0, t1, sa, sb, t2;
  fp_mul(t0, a.c0, b.c0);
  fp_mul(t1, a.c1, b.c1);
  fp_add(sa, a.c0, a.c1);
  fp_add(sb, b.c0, b.c1);
  fp_mul(t2, sa, sb);
  fp_sub(r.c0, t0, t1);
  fp_sub(t2, t2, t0);
  fp_sub(r.c1, t2, t1);
}
// (a0+a1)(a0-a1), 2 a0 a1: 2 Fp products
HD void fp2_sqr(fp2 &r, const fp2 &a) {
  fp s, d, m;
  fp_add(s, a.c0, a.c1);
  fp_sub(d, a.c0, a.c1);
  fp_mul(m, a.c0, a.c1);
  fp_mul(r.c0, s, d);
  fp_add(r.c1, m, m);
}
HD void fp2_mul_fp(fp2 &r, const fp2 &a, const fp &b) {
  fp_mul(r.c0, a.c0, b);
  fp_mul(r.c1, a.c1, b);
}
// times xi = 1 + u
HD void fp2_mul_xi(fp2 &r, const fp2 &a) {
  fp t0, t1;
  fp_sub(t0, a.c0, a.c1);
  fp_add(t1, a.c0, a.c1);
  r.c0 = t0;
  r.c1 = t1;
}
HD void fp2_mul3(fp2 &r, const fp2 &a) {
  fp_mul3(r.c0, a.c0);
  fp_mul3(r.c1, a.c1);
}
HD void fp2_inv(fp2 &r, const fp2 &a) {
  fp t0, t1, n;
  fp_sqr(t0, a.c0);
  fp_sqr(t1, a.c1);
  fp_add(n, t0, t1);
  fp_inv(n, n);
  fp_mul(r.c0, a.c0, n);
  fp_mul(t1, a.c1, n);
  fp_neg(r.c1, t1);
}
HD bool fp2_lex_largest(const fp2 &a) {
  return fp_is_zero(a.c1) ? fp_lex_largest(a.c0) : fp_lex_largest(a.c1);
}
// RFC 9380 sgn0 for m = 2
HD uint32_t fp2_sgn0(const fp2 &a) {
  uint32_t s0 = fp_parity(a.c0);
  uint32_t z0 = fp_is_zero(a.c0);
  uint32_t s1 = fp_parity(a.c1);
  return s0 | (z0 & s1);
}

// Square root in Fp2 (complex method, two Fp exponentiations).
// Given gamma = sqrt(N(a)) in Fp (precomputed by the caller, who also decided that
// a is a square), returns a root of a.  Derivation in DESIGN.md §Fp2 sqrt.
HD void fp2_sqrt_given_norm_root(fp2 &r, const fp2 &a, const fp &gamma) {
  const fp inv2 = fp_const(k::INV2_M);
  fp delta, t, x0, x0sq, tmp;
  fp_add(delta, a.c0, gamma);
  fp_mul(delta, delta, inv2);
  if (fp_is_zero(delta)) {  // only when a1 == 0 and gamma == -a0
    fp_sub(delta, a.c0, gamma);
    fp_mul(delta, delta, inv2);
  }
  fp_pow(t, delta, k::EXP_PM3D4);
  fp_mul(x0, delta, t);
  fp_sqr(x0sq, x0);
  fp half_a1t;
  fp_mul(tmp, a.c1, t);
  fp_mul(half_a1t, tmp, inv2);
  if (fp_eq(x0sq, delta)) {  // delta is a square: (x0, a1 t / 2)
    r.c0 = x0;
    r.c1 = half_a1t;
  } else {  // delta non-square: (-a1 t / 2, delta t)
    fp_neg(r.c0, half_a1t);
    r.c1 = x0;
  }
}
// returns true iff a is a square (then r is a root)
HD bool fp2_sqrt(fp2 &r, const fp2 &a) {
  if (fp2_is_zero(a)) {
    fp2_zero(r);
    return true;
  }
  fp n, t, gamma;
  fp_sqr(n, a.c0);
  fp_sqr(t, a.c1);
  fp_add(n, n, t);
  if (!fp_sqrt(gamma, n)) return false;
  fp2_sqrt_given_norm_root(r, a, gamma);
  fp2 chk;
  fp2_sqr(chk, r);
  return fp2_eq(chk, a);
}

// ---------------------------------------------------------------- Fp6
HD void fp6_zero(fp6 &r) {
  fp2_zero(r.c0);
  fp2_zero(r.c1);
  fp2_zero(r.c2);
}
HD void fp6_one(fp6 &r) {
  fp2_one(r.c0);
  fp2_zero(r.c1);
  fp2_zero(r.c2);
}
HD void fp6_add(fp6 &r, const fp6 &a, const fp6 &b) {
  fp2_add(r.c0, a.c0, b.c0);
  fp2_add(r.c1, a.c1, b.c1);
  fp2_add(r.c2, a.c2, b.c2);
}
HD void fp6_sub(fp6 &r, const fp6 &a, const fp6 &b) {
  fp2_sub(r.c0, a.c0, b.c0);
  fp2_sub(r.c1, a.c1, b.c1);
  fp2_sub(r.c2, a.c2, b.c2);
}
HD void fp6_neg(fp6 &r, const fp6 &a) {
  fp2_neg(r.c0, a.c0);
  fp2_neg(r.c1, a.c1);
  fp2_neg(r.c2, a.c2);
}
// times v: (c0, c1, c2) -> (xi c2, c0, c1)
HD void fp6_mul_v(fp6 &r, const fp6 &a) {
  fp2 t;
  fp2_mul_xi(t, a.c2);
  r.c2 = a.c1;
  r.c1 = a.c0;
  r.c0 = t;
}
// Karatsuba: 6 Fp2 products
HD void fp6_mul(fp6 &r, const fp6 &a, const fp6 &b) {
  fp2 t0, t1, t2, s0, s1, c0, c1, c2;
  fp2_mul(t0, a.c0, b.c0);
  fp2_mul(t1, a.c1, b.c1);
  fp2_mul(t2, a.c2, b.c2);
  fp2_add(s0, a.c1, a.c2);
  fp2_add(s1, b.c1, b.c2);
  fp2_mul(c0, s0, s1);
  fp2_sub(c0, c0, t1);
  fp2_sub(c0, c0, t2);
  fp2_mul_xi(c0, c0);
  fp2_add(c0, c0, t0);
  fp2_add(s0, a.c0, a.c1);
  fp2_add(s1, b.c0, b.c1);
  fp2_mul(c1, s0, s1);
  fp2_sub(c1, c1, t0);
  fp2_sub(c1, c1, t1);
  fp2_mul_xi(s0, t2);
  fp2_add(c1, c1, s0);
  fp2_add(s0, a.c0, a.c2);
  fp2_add(s1, b.c0, b.c2);
  fp2_mul(c2, s0, s1);
  fp2_sub(c2, c2, t0);
  fp2_sub(c2, c2, t2);
  fp2_add(c2, c2, t1);
  r.c0 = c0;
  r.c1 = c1;
  r.c2 = c2;
}
// a * (b0 + b1 v): 5 Fp2 products
HD void fp6_mul_01(fp6 &r, const fp6 &a, const fp2 &b0, const fp2 &b1) {
  fp2 t0, t1, s0, s1, c0, c1, c2;
  fp2_mul(t0, a.c0, b0);
  fp2_mul(t1, a.c1, b1);
  fp2_add(s0, a.c1, a.c2);
  fp2_mul(c0, s0, b1);
  fp2_sub(c0, c0, t1);
  fp2_mul_xi(c0, c0);
  fp2_add(c0, c0, t0);
  fp2_add(s0, a.c0, a.c1);
  fp2_add(s1, b0, b1);
  fp2_mul(c1, s0, s1);
  fp2_sub(c1, c1, t0);
  fp2_sub(c1, c1, t1);
  fp2_add(s0, a.c0, a.c2);
  fp2_mul(c2, s0, b0);
  fp2_sub(c2, c2, t0);
  fp2_add(c2, c2, t1);
  r.c0 = c0;
  r.c1 = c1;
  r.c2 = c2;
}
// a * (b1 v): 3 Fp2 products
HD void fp6_mul_1(fp6 &r, const fp6 &a, const fp2 &b1) {
  fp2 c0, c1, c2;
  fp2_mul(c0, a.c2, b1);
  fp2_mul_xi(c0, c0);
  fp2_mul(c1, a.c0, b1);
  fp2_mul(c2, a.c1, b1);
  r.c0 = c0;
  r.c1 = c1;
  r.c2 = c2;
}
HD void fp6_inv(fp6 &r, const fp6 &a) {
  fp2 c0, c1, c2, t, s;
  fp2_sqr(c0, a.c0);
  fp2_mul(t, a.c1, a.c2);
  fp2_mul_xi(t, t);
  fp2_sub(c0, c0, t);
  fp2_sqr(c1, a.c2);
  fp2_mul_xi(c1, c1);
  fp2_mul(t, a.c0, a.c1);
  fp2_sub(c1, c1, t);
  fp2_sqr(c2, a.c1);
  fp2_mul(t, a.c0, a.c2);
  fp2_sub(c2, c2, t);
  fp2_mul(t, a.c2, c1);
  fp2_mul(s, a.c1, c2);
  fp2_add(t, t, s);
  fp2_mul_xi(t, t);
  fp2_mul(s, a.c0, c0);
  fp2_add(t, t, s);
  fp2_inv(t, t);
  fp2_mul(r.c0, c0, t);
  fp2_mul(r.c1, c1, t);
  fp2_mul(r.c2, c2, t);
}

// ---------------------------------------------------------------- Fp12
HD void fp12_one(fp12 &r) {
  fp6_one(r.c0);
  fp6_zero(r.c1);
}
HD bool fp12_is_one(const fp12 &a) {
  fp2 one;
  fp2_one(one);
  return fp2_eq(a.c0.c0, one) && fp2_is_zero(a.c0.c1) && fp2_is_zero(a.c0.c2) &&
         fp2_is_zero(a.c1.c0) && fp2_is_zero(a.c1.c1) && fp2_is_zero(a.c1.c2);
}
HD void fp12_conj(fp12 &r, const fp12 &a) {
  r.c0 = a.c0;
  fp6_neg(r.c1, a.c1);
}
// Karatsuba over Fp6: 18 Fp2 products
HD void fp12_mul(fp12 &r, const fp12 &a, const fp12 &b) {
  fp6 t0, t1, s0, s1;
  fp6_mul(t0, a.c0, b.c0);
  fp6_mul(t1, a.c1, b.c1);
  fp6_add(s0, a.c0, a.c1);
  fp6_add(s1, b.c0, b.c1);
  fp6_mul(s0, s0, s1);
  fp6_sub(s0, s0, t0);
  fp6_sub(r.c1, s0, t1);
  fp6_mul_v(t1, t1);
  fp6_add(r.c0, t0, t1);
}
// complex squaring: 2 Fp6 products
HD void fp12_sqr(fp12 &r, const fp12 &a) {
  fp6 t, s0, s1, vt;
  fp6_mul(t, a.c0, a.c1);
  fp6_add(s0, a.c0, a.c1);
  fp6_mul_v(s1, a.c1);
  fp6_add(s1, s1, a.c0);
  fp6_mul(s0, s0, s1);
  fp6_sub(s0, s0, t);
  fp6_mul_v(vt, t);
  fp6_sub(r.c0, s0, vt);
  fp6_add(r.c1, t, t);
}
// multiply by a Miller-loop line  l0 + l2 w^2 + l3 w^3  =  (l0 + l2 v) + (l3 v) w
HD void fp12_mul_line(fp12 &r, const fp12 &a, const fp2 &l0, const fp2 &l2, const fp2 &l3) {
  fp6 t0, t1, s;
  fp6_mul_01(t0, a.c0, l0, l2);
  fp6_mul_1(t1, a.c1, l3);
  fp6_add(s, a.c0, a.c1);
  fp2 l23;
  fp2_add(l23, l2, l3);
  fp6_mul_01(s, s, l0, l23);
  fp6_sub(s, s, t0);
  fp6_sub(r.c1, s, t1);
  fp6_mul_v(t1, t1);
  fp6_add(r.c0, t0, t1);
}
HD void fp12_inv(fp12 &r, const fp12 &a) {
  fp6 t0, t1;
  fp6_mul(t0, a.c0, a.c0);
  fp6_mul(t1, a.c1, a.c1);
  fp6_mul_v(t1, t1);
  fp6_sub(t0, t0, t1);
  fp6_inv(t0, t0);
  fp6_mul(r.c0, a.c0, t0);
  fp6_mul(t1, a.c1, t0);
  fp6_neg(r.c1, t1);
}
// Frobenius x -> x^p.  Coefficient of w^k: a0(k0) b0(k1) a1(k2) b1(k3) a2(k4) b2(k5).
HD void fp12_frob(fp12 &r, const fp12 &a) {
  fp2 t;
  fp2_conj(r.c0.c0, a.c0.c0);
  fp2_conj(t, a.c1.c0);
  fp2_mul(r.c1.c0, t, fp2_const(k::FROB1_1_C0, k::FROB1_1_C1));
  fp2_conj(t, a.c0.c1);
  fp2_mul(r.c0.c1, t, fp2_const(k::FROB1_2_C0, k::FROB1_2_C1));
  fp2_conj(t, a.c1.c1);
  fp2_mul(r.c1.c1, t, fp2_const(k::FROB1_3_C0, k::FROB1_3_C1));
  fp2_conj(t, a.c0.c2);
  fp2_mul(r.c0.c2, t, fp2_const(k::FROB1_4_C0, k::FROB1_4_C1));
  fp2_conj(t, a.c1.c2);
  fp2_mul(r.c1.c2, t, fp2_const(k::FROB1_5_C0, k::FROB1_5_C1));
}
HD void fp12_frob2(fp12 &r, const fp12 &a) {
  r.c0.c0 = a.c0.c0;
  fp2_mul_fp(r.c1.c0, a.c1.c0, fp_const(k::FROB2_1_M));
  fp2_mul_fp(r.c0.c1, a.c0.c1, fp_const(k::FROB2_2_M));
  fp2_mul_fp(r.c1.c1, a.c1.c1, fp_const(k::FROB2_3_M));
  fp2_mul_fp(r.c0.c2, a.c0.c2, fp_const(k::FROB2_4_M));
  fp2_mul_fp(r.c1.c2, a.c1.c2, fp_const(k::FROB2_5_M));
}

}  // namespace gbls
