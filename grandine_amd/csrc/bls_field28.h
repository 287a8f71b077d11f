// Radix-2^28 arithmetic over the BLS12-381 base field: the next field layer,
// used so far by the (p-3)/4 exponentiation (hash_to_G2's SSWU, decompression square roots)
// and the GBLS_ML_R28 k_ml_group28; tools/ubench/r28_bench.hip measured its product at 1.40x
// the engine's product per lane on MI355X.
//
// An element is 14 limbs of 28 bits in Montgomery form with R = 2^392.  A column of the
// product-scanning Montgomery product holds at most 28 terms (42 for a dual product), so with
// limbs < 2^29 every term is < 2^58 and the column fits one 64-bit accumulator: one
// v_mad_u64_u32 per term and no carry word (the engine's 32-bit limbs need a mad + addc pair).
// R/p ~ 2^11.3, so the REDC bound T < R p holds for inputs up to ~35 p (dual) and outputs are
// < p (1 + T / (R p)) ~ 1.01 p: no final subtraction.
//
// Limb and value contract:
//   normalized: every limb < 2^28 (outputs of mul, mul2, norm, sub, from_fp);
//   mul/mul2 inputs: limbs < 2^29 (one add_lazy of two normalized elements), values < 32 p;
//   sub(a, b) = norm(4p + a - b) needs b normalized and < 4p + a (4p is stored with every limb
//   but the top in [2^28 - 1, 2^29), so no lower limb borrows; the top limb wraps back);
//   neg_lazy(a) = 4p - a needs a < 2p.
// canon() gives the unique representative in [0, p) (values < 16 p).
#pragma once
// needs bls_field.h (struct fp, HD) included first; bls_field.h itself includes this header
// for its (p-3)/4 exponentiation (unless GBLS_POW_ENGINE)
#include <stdint.h>

// Host builds with GBLS_R28_CHECK (tests/native/host_harness.cpp) abort when an operation's limb
// contract above is broken: a product operand limb >= 2^29, a biased difference with a negative
// limb, a value >= 2^392 where a reduction expects less.  Device code never checks.
#if !defined(__HIP_DEVICE_COMPILE__) && defined(GBLS_R28_CHECK)
#include <stdlib.h>
#define R28_CHECK(c) \
  do {               \
    if (!(c)) abort(); \
  } while (0)
#else
#define R28_CHECK(c) ((void)0)
#endif

namespace gbls {
namespace r28 {

struct fe {
  uint32_t l[14];
};
struct fe2 {
  fe c0, c1;
};

constexpr uint32_t kMask = 0x0fffffff;
constexpr uint32_t kPinv = 0x0ffcfffd;  // -p^-1 mod 2^28

#define GBLS_R28_P                                                                              \
  0xfffaaab, 0xfefffff, 0x3ffffb9, 0xfffeb15, 0x6241eab, 0xa0f6b0f, 0xf6730d2, 0xf38512b,        \
      0x4774b84, 0x4bacd76, 0xba7b643, 0xe69a4b1, 0x1ea397f, 0x1a011
// 4p, every limb but the top rebalanced into [2^28 - 1, 2^29)
#define GBLS_R28_BIAS4P                                                                         \
  0x1ffeaaac, 0x1fbffffe, 0x1ffffee6, 0x1fffac53, 0x18907aae, 0x183dac3c, 0x1d9cc349,            \
      0x1ce144ae, 0x11dd2e12, 0x12eb35d8, 0x1e9ed90c, 0x19a692c5, 0x17a8e5fe, 0x68043
// 8p, every limb but the top rebalanced into [2^28 - 1, 2^29)
#define GBLS_R28_BIAS8P                                                                         \
  0x1ffd5558, 0x1f7ffffe, 0x1ffffdce, 0x1fff58a8, 0x1120f55e, 0x107b587a, 0x1b398694,           \
      0x19c2895e, 0x13ba5c26, 0x15d66bb1, 0x1d3db219, 0x134d258c, 0x1f51cbfe, 0xd0087
// 2^400 mod p: x 2^384 (engine form) times this, over R = 2^392, is x 2^392
#define GBLS_R28_CIN                                                                            \
  0x80e6299, 0x3500034, 0xeb12856, 0xdeb2699, 0xc988670, 0x4ef6697, 0x70983e8, 0xa4e6fe9,        \
      0x3e8a053, 0xecf271e, 0xc20d323, 0x6eb6385, 0x47f1286, 0x156da
// 2^384 mod p: x 2^392 times this, over R, is x 2^384
#define GBLS_R28_COUT                                                                           \
  0x2fffd, 0x900000, 0xc000276, 0xbc40, 0x8baebf4, 0x5753c75, 0x55f4898, 0x7052574, 0x7ce5853,   \
      0x56ec6d7, 0x71a97a2, 0xe4935c0, 0xec3fa80, 0x15f65

// (sum over the NP pairs x_k y_k) / 2^392 mod p, product scanning
template <int NP>
HD void mul_n(fe &r, const fe *const *x, const fe *const *y) {
  constexpr uint32_t P[14] = {GBLS_R28_P};
  uint32_t m[14], t[14];
  uint64_t acc = 0;
  for (int q = 0; q < NP; q++)
    for (int i = 0; i < 14; i++) R28_CHECK(x[q]->l[i] < (1u << 29) && y[q]->l[i] < (1u << 29));
#pragma unroll
  for (int k = 0; k < 27; k++) {
#pragma unroll
    for (int i = 0; i < 14; i++) {
      const int j = k - i;
      if (j >= 0 && j < 14) {
#pragma unroll
        for (int q = 0; q < NP; q++) acc += (uint64_t)x[q]->l[i] * y[q]->l[j];
      }
    }
#pragma unroll
    for (int i = 0; i < 14; i++) {
      const int j = k - i;
      if (i < k && j >= 0 && j < 14) acc += (uint64_t)m[i] * P[j];
    }
    if (k < 14) {
      m[k] = ((uint32_t)acc * kPinv) & kMask;
      acc += (uint64_t)m[k] * P[0];
    } else {
      t[k - 14] = (uint32_t)acc & kMask;
    }
    acc >>= 28;
  }
  t[13] = (uint32_t)acc;
#pragma unroll
  for (int i = 0; i < 14; i++) r.l[i] = t[i];
}
#if defined(__HIP_DEVICE_COMPILE__)
constexpr uint32_t kP28[14] = {GBLS_R28_P};
#include "bls_fpmul28_gen.h"
#endif
HD void mul(fe &r, const fe &a, const fe &b) {
#if defined(__HIP_DEVICE_COMPILE__)
  fe_mul_dev(r, a, b);
#else
  const fe *x[1] = {&a}, *y[1] = {&b};
  mul_n<1>(r, x, y);
#endif
}
// a^2: the cross terms once against the doubled limbs (105 product terms + the reduction's
// 196, against 392 for mul(a, a)); limbs of a < 2^29
HD void sqr(fe &r, const fe &a) {
#if defined(__HIP_DEVICE_COMPILE__)
  fe_sqr_dev(r, a);
#else
  const fe *x[1] = {&a}, *y[1] = {&a};
  mul_n<1>(r, x, y);
#endif
}
// a b + c d in one reduction
HD void mul2(fe &r, const fe &a, const fe &b, const fe &c, const fe &d) {
#if defined(__HIP_DEVICE_COMPILE__)
  fe_mul2_dev(r, a, b, c, d);
#else
  const fe *x[2] = {&a, &c}, *y[2] = {&b, &d};
  mul_n<2>(r, x, y);
#endif
}

// x0 y0 + ... + x5 y5 in one reduction (one operand of each pair normalized, the other with
// limbs < 2^29; values < 34 p^2 in all: output < 1.02 p)
HD void mul6(fe &r, const fe &x0, const fe &y0, const fe &x1, const fe &y1, const fe &x2, const fe &y2,
             const fe &x3, const fe &y3, const fe &x4, const fe &y4, const fe &x5, const fe &y5) {
#if defined(__HIP_DEVICE_COMPILE__)
  fe_mul6_dev(r, x0, y0, x1, y1, x2, y2, x3, y3, x4, y4, x5, y5);
#else
  const fe *x[6] = {&x0, &x1, &x2, &x3, &x4, &x5}, *y[6] = {&y0, &y1, &y2, &y3, &y4, &y5};
  mul_n<6>(r, x, y);
#endif
}

HD void mul4(fe &r, const fe &x0, const fe &y0, const fe &x1, const fe &y1, const fe &x2, const fe &y2,
             const fe &x3, const fe &y3) {
#if defined(__HIP_DEVICE_COMPILE__)
  fe_mul4_dev(r, x0, y0, x1, y1, x2, y2, x3, y3);
#else
  const fe *x[4] = {&x0, &x1, &x2, &x3}, *y[4] = {&y0, &y1, &y2, &y3};
  mul_n<4>(r, x, y);
#endif
}

HD void norm(fe &a) {
#pragma unroll
  for (int i = 0; i < 13; i++) {
    a.l[i + 1] += a.l[i] >> 28;
    a.l[i] &= kMask;
  }
}
// limbwise, no carries: limbs < 2^29 from normalized inputs (a product operand)
HD void add_lazy(fe &r, const fe &a, const fe &b) {
#pragma unroll
  for (int i = 0; i < 14; i++) r.l[i] = a.l[i] + b.l[i];
}
HD void add(fe &r, const fe &a, const fe &b) {
  add_lazy(r, a, b);
  norm(r);
}
// 4p + a - b, normalized (b < 4p, normalized)
HD void sub(fe &r, const fe &a, const fe &b) {
  constexpr uint32_t B[14] = {GBLS_R28_BIAS4P};
  for (int i = 0; i < 13; i++) R28_CHECK(b.l[i] <= B[i]);
#pragma unroll
  for (int i = 0; i < 14; i++) r.l[i] = B[i] + a.l[i] - b.l[i];
  norm(r);
  R28_CHECK(r.l[13] < (1u << 28));
}
// 4p - a (a < 2p, normalized): limbs < 2^29, a product operand without normalization
HD void neg_lazy(fe &r, const fe &a) {
  constexpr uint32_t B[14] = {GBLS_R28_BIAS4P};
#pragma unroll
  for (int i = 0; i < 14; i++) r.l[i] = B[i] - a.l[i];
}

// a - p if a >= p (a normalized); returns 1 if it subtracted
HD uint32_t sub_p_if_geq(fe &a) {
  constexpr uint32_t P[14] = {GBLS_R28_P};
  fe d;
  int32_t borrow = 0;
#pragma unroll
  for (int i = 0; i < 14; i++) {
    int32_t v = (int32_t)a.l[i] - (int32_t)P[i] + borrow;
    borrow = v >> 28;  // 0 or -1 (arithmetic shift)
    d.l[i] = (uint32_t)v & kMask;
  }
  const uint32_t ge = borrow == 0;
#pragma unroll
  for (int i = 0; i < 14; i++) a.l[i] = ge ? d.l[i] : a.l[i];
  return ge;
}
// the representative in [0, p) of a value < 16 p
HD void canon(fe &a) {
  norm(a);
  for (int s = 0; s < 15; s++)
    if (!sub_p_if_geq(a)) break;
}
HD bool is_zero(const fe &a) {
  fe t = a;
  canon(t);
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < 14; i++) o |= t.l[i];
  return o == 0;
}

// engine form (12 x 32-bit limbs, x 2^384 mod p, < 2^384) <-> radix-2^28 form (x 2^392)
HD void repack_in(fe &r, const fp &a) {
#pragma unroll
  for (int i = 0; i < 14; i++) {
    const int bit = 28 * i, w = bit >> 5, s = bit & 31;
    uint32_t v = a.l[w] >> s;
    if (s > 4 && w + 1 < 12) v |= a.l[w + 1] << (32 - s);
    r.l[i] = v & kMask;
  }
}
HD void repack_out(fp &r, const fe &a) {
  uint64_t buf = 0;
  int have = 0, w = 0;
#pragma unroll
  for (int i = 0; i < 14; i++) {
    buf |= (uint64_t)a.l[i] << have;
    have += 28;
    if (have >= 32 && w < 12) {
      r.l[w++] = (uint32_t)buf;
      buf >>= 32;
      have -= 32;
    }
  }
  if (w < 12) r.l[w] = (uint32_t)buf;
}
HD void from_fp(fe &r, const fp &a) {
  constexpr fe C = {{GBLS_R28_CIN}};
  fe t;
  repack_in(t, a);
  mul(r, t, C);
}
HD void to_fp(fp &r, const fe &a) {
  constexpr fe C = {{GBLS_R28_COUT}};
  fe t;
  mul(t, a, C);
  canon(t);
  repack_out(r, t);
}

// a - q p for q = floor(top limb / (p_top + 1)) <= a / p: a normalized (< 2^392) -> < 1.03 p
HD void wred(fe &a) {
  constexpr uint32_t P[14] = {GBLS_R28_P};
  for (int i = 0; i < 14; i++) R28_CHECK(a.l[i] < (1u << 28));
  const uint32_t q = a.l[13] / 0x1a012u;
  int64_t c = 0;
#pragma unroll
  for (int i = 0; i < 14; i++) {
    c += (int64_t)a.l[i] - (int64_t)q * P[i];
    a.l[i] = (uint32_t)c & kMask;
    c >>= 28;
  }
}
// 8p + a - b, normalized and weakly reduced (< 1.03 p): b normalized, < 8p + a
HD void sub_r(fe &r, const fe &a, const fe &b) {
  constexpr uint32_t B[14] = {GBLS_R28_BIAS8P};
  for (int i = 0; i < 13; i++) R28_CHECK(b.l[i] <= B[i]);
#pragma unroll
  for (int i = 0; i < 14; i++) r.l[i] = B[i] + a.l[i] - b.l[i];
  norm(r);
  wred(r);
}

// ---------------------------------------------- lazy point arithmetic (bls_curve28.h)
// The doubling formulas add and subtract up to three terms before a product or an output:
// instead of reducing after each step (sub_r / add + wred: norm + wred, ~115 VALU per Fp), a
// combination is formed limbwise against a bias, normalized once and weakly reduced only when
// its consumer needs it.
struct bias_t {
  uint32_t l[14];
};
// m p with every limb but the top raised by b (2^28 - 1) (borrowed from the limb above): a
// subtrahend with limbs <= b (2^28 - 1) leaves every limb nonnegative.  make_bias(4, 1) and
// make_bias(8, 1) are GBLS_R28_BIAS4P / BIAS8P (static_assert below).
constexpr bias_t make_bias(uint32_t m, uint32_t b) {
  const uint32_t P[14] = {GBLS_R28_P};
  bias_t r{};
  uint64_t c = 0;
  for (int i = 0; i < 14; i++) {
    c += (uint64_t)m * P[i];
    r.l[i] = (uint32_t)(c & kMask);
    c >>= 28;
  }
  for (int i = 0; i < 13; i++) {
    r.l[i] += b << 28;
    r.l[i + 1] -= b;
  }
  return r;
}
constexpr bool bias_is(const bias_t &a, const bias_t &b) {
  for (int i = 0; i < 14; i++)
    if (a.l[i] != b.l[i]) return false;
  return true;
}
static_assert(bias_is(make_bias(4, 1), bias_t{{GBLS_R28_BIAS4P}}), "bias generator");
static_assert(bias_is(make_bias(8, 1), bias_t{{GBLS_R28_BIAS8P}}), "bias generator");

// a + b, normalized, not reduced (a, b normalized)
HD void add_n(fe &r, const fe &a, const fe &b) { add(r, a, b); }
// k a, normalized, not reduced (a normalized, k <= 15)
HD void mulk_n(fe &r, const fe &a, uint32_t k) {
#pragma unroll
  for (int i = 0; i < 14; i++) r.l[i] = k * a.l[i];
  norm(r);
}
// k a weakly reduced (< 1.03 p): a normalized, k a < 2^392
HD void mulk_r(fe &r, const fe &a, uint32_t k) {
  mulk_n(r, a, k);
  wred(r);
}
// S (a - K1 b - K2 c) weakly reduced (< 1.03 p): formed limbwise against 16 p raised for
// K1 + K2 normalized subtrahend limbs, normalized once; a, b, c normalized,
// K1 b + K2 c < 16 p + a, S (K1 + K2 + 2) <= 15 (every limb < 2^32)
template <uint32_t S, uint32_t K1, uint32_t K2>
HD void lin_r(fe &r, const fe &a, const fe &b, const fe &c) {
  static_assert(S * (K1 + K2 + 2) <= 15, "limb bound");
  constexpr bias_t B = make_bias(16, K1 + K2);
  for (int i = 0; i < 13; i++) R28_CHECK(K1 * b.l[i] + K2 * c.l[i] <= B.l[i]);
#pragma unroll
  for (int i = 0; i < 14; i++) r.l[i] = S * (B.l[i] + a.l[i] - K1 * b.l[i] - K2 * c.l[i]);
  norm(r);
  R28_CHECK(r.l[13] < (1u << 28));
  wred(r);
}
// S (a - K b), the same
template <uint32_t S, uint32_t K>
HD void lin_r(fe &r, const fe &a, const fe &b) {
  static_assert(S * (K + 2) <= 15, "limb bound");
  constexpr bias_t B = make_bias(16, K);
  for (int i = 0; i < 13; i++) R28_CHECK(K * b.l[i] <= B.l[i]);
#pragma unroll
  for (int i = 0; i < 14; i++) r.l[i] = S * (B.l[i] + a.l[i] - K * b.l[i]);
  norm(r);
  R28_CHECK(r.l[13] < (1u << 28));
  wred(r);
}
// a - K b; S (a - b - c)
template <uint32_t K>
HD void subk_r(fe &r, const fe &a, const fe &b) {
  lin_r<1, K>(r, a, b);
}
template <uint32_t S>
HD void sub2_r(fe &r, const fe &a, const fe &b, const fe &c) {
  lin_r<S, 1, 1>(r, a, b, c);
}

// ------------------------------------------------------------------ Fp2 = Fp[u] / (u^2 + 1)
// a: limbs < 2^29 (a lazy sum of normalized elements), value < 5p; b: normalized, < 5p;
// output < 1.03 p
HD void fe2_mul(fe2 &r, const fe2 &a, const fe2 &b) {
  constexpr uint32_t B[14] = {GBLS_R28_BIAS8P};
  for (int i = 0; i < 13; i++) R28_CHECK(b.c1.l[i] <= B[i]);
  R28_CHECK(b.c1.l[13] <= B[13]);
  fe nb1, c0;
#pragma unroll
  for (int i = 0; i < 14; i++) nb1.l[i] = B[i] - b.c1.l[i];
  mul2(c0, a.c0, b.c0, a.c1, nb1);
  mul2(r.c1, a.c0, b.c1, a.c1, b.c0);
  r.c0 = c0;
}
// (a0 + a1)(a0 - a1), 2 a0 a1
HD void fe2_sqr(fe2 &r, const fe2 &a) {
  for (int i = 0; i < 14; i++) R28_CHECK(a.c0.l[i] < (1u << 28) && a.c1.l[i] < (1u << 28));
  fe s, d, t;
  add_lazy(s, a.c0, a.c1);
  sub(d, a.c0, a.c1);
  add_lazy(t, a.c1, a.c1);
  mul(r.c1, a.c0, t);
  mul(r.c0, s, d);
}
HD void fe2_add(fe2 &r, const fe2 &a, const fe2 &b) {
  add(r.c0, a.c0, b.c0);
  add(r.c1, a.c1, b.c1);
}
HD void fe2_sub(fe2 &r, const fe2 &a, const fe2 &b) {
  sub(r.c0, a.c0, b.c0);
  sub(r.c1, a.c1, b.c1);
}
HD void fe2_mul_fe(fe2 &r, const fe2 &a, const fe &b) {
  mul(r.c0, a.c0, b);
  mul(r.c1, a.c1, b);
}
// times xi = 1 + u
HD void fe2_mul_xi(fe2 &r, const fe2 &a) {
  fe t0, t1;
  sub(t0, a.c0, a.c1);
  add(t1, a.c0, a.c1);
  r.c0 = t0;
  r.c1 = t1;
}

// ---------------------------------------------- sparse Miller-loop products (k_ml_group)
// Every coefficient a routine returns is normalized and < 1.1 p ("S"); routines take S (or
// normalized sums of two S) and follow the engine's formulas (bls_pairing.h sp_mul_sp,
// fp6_mul_01, fp6_mul_1, fp12_mul_034), with each subtraction weakly reduced.
struct fe6 {
  fe2 c0, c1, c2;
};
struct fe12 {
  fe6 c0, c1;
};
struct sp {  // a0 + a2 w^2 + a3 w^3
  fe2 a0, a2, a3;
};

HD void fe2_add_lazy(fe2 &r, const fe2 &a, const fe2 &b) {
  add_lazy(r.c0, a.c0, b.c0);
  add_lazy(r.c1, a.c1, b.c1);
}
HD void fe2_sub_r(fe2 &r, const fe2 &a, const fe2 &b) {
  sub_r(r.c0, a.c0, b.c0);
  sub_r(r.c1, a.c1, b.c1);
}
// a + b, weakly reduced
HD void fe2_add_r(fe2 &r, const fe2 &a, const fe2 &b) {
  add(r.c0, a.c0, b.c0);
  add(r.c1, a.c1, b.c1);
  wred(r.c0);
  wred(r.c1);
}
// the lazy combinations (bls_curve28.h), per coordinate
HD void fe2_add_n(fe2 &r, const fe2 &a, const fe2 &b) {
  add_n(r.c0, a.c0, b.c0);
  add_n(r.c1, a.c1, b.c1);
}
HD void fe2_mulk_n(fe2 &r, const fe2 &a, uint32_t k) {
  mulk_n(r.c0, a.c0, k);
  mulk_n(r.c1, a.c1, k);
}
HD void fe2_mulk_r(fe2 &r, const fe2 &a, uint32_t k) {
  mulk_r(r.c0, a.c0, k);
  mulk_r(r.c1, a.c1, k);
}
template <uint32_t K>
HD void fe2_subk_r(fe2 &r, const fe2 &a, const fe2 &b) {
  subk_r<K>(r.c0, a.c0, b.c0);
  subk_r<K>(r.c1, a.c1, b.c1);
}
template <uint32_t S>
HD void fe2_sub2_r(fe2 &r, const fe2 &a, const fe2 &b, const fe2 &c) {
  sub2_r<S>(r.c0, a.c0, b.c0, c.c0);
  sub2_r<S>(r.c1, a.c1, b.c1, c.c1);
}
template <uint32_t S, uint32_t K>
HD void fe2_lin_r(fe2 &r, const fe2 &a, const fe2 &b) {
  lin_r<S, K>(r.c0, a.c0, b.c0);
  lin_r<S, K>(r.c1, a.c1, b.c1);
}
template <uint32_t S, uint32_t K1, uint32_t K2>
HD void fe2_lin_r(fe2 &r, const fe2 &a, const fe2 &b, const fe2 &c) {
  lin_r<S, K1, K2>(r.c0, a.c0, b.c0, c.c0);
  lin_r<S, K1, K2>(r.c1, a.c1, b.c1, c.c1);
}
HD void fe2_zero(fe2 &r) {
#pragma unroll
  for (int i = 0; i < 14; i++) r.c0.l[i] = r.c1.l[i] = 0;
}
// times xi = 1 + u
HD void fe2_mul_xi_r(fe2 &r, const fe2 &a) {
  fe t0, t1;
  sub_r(t0, a.c0, a.c1);
  add(t1, a.c0, a.c1);
  wred(t1);
  r.c0 = t0;
  r.c1 = t1;
}
HD void fe6_add(fe6 &r, const fe6 &a, const fe6 &b) {  // normalized, not reduced
  fe2_add_lazy(r.c0, a.c0, b.c0);
  fe2_add_lazy(r.c1, a.c1, b.c1);
  fe2_add_lazy(r.c2, a.c2, b.c2);
  norm(r.c0.c0), norm(r.c0.c1), norm(r.c1.c0), norm(r.c1.c1), norm(r.c2.c0), norm(r.c2.c1);
}
HD void fe6_sub_r(fe6 &r, const fe6 &a, const fe6 &b) {
  fe2_sub_r(r.c0, a.c0, b.c0);
  fe2_sub_r(r.c1, a.c1, b.c1);
  fe2_sub_r(r.c2, a.c2, b.c2);
}

// (a0 + a2 w^2 + a3 w^3)(b0 + b2 w^2 + b3 w^3): 6 Fp2 products
HD void sp_mul_sp(fe12 &r, const sp &a, const sp &b) {
  fe2 t0, t2, t3, sa, sb, u;
  fe2_mul(t0, a.a0, b.a0);
  fe2_mul(t2, a.a2, b.a2);
  fe2_mul(t3, a.a3, b.a3);
  fe2_mul_xi_r(u, t3);
  fe2_add_r(r.c0.c0, t0, u);
  fe2_zero(r.c1.c0);
  fe2_add_lazy(sa, a.a0, a.a2);
  fe2_add_lazy(sb, b.a0, b.a2);
  norm(sb.c0), norm(sb.c1);
  fe2_mul(u, sa, sb);
  fe2_sub_r(u, u, t0);
  fe2_sub_r(r.c0.c1, u, t2);
  fe2_add_lazy(sa, a.a0, a.a3);
  fe2_add_lazy(sb, b.a0, b.a3);
  norm(sb.c0), norm(sb.c1);
  fe2_mul(u, sa, sb);
  fe2_sub_r(u, u, t0);
  fe2_sub_r(r.c1.c1, u, t3);
  r.c0.c2 = t2;
  fe2_add_lazy(sa, a.a2, a.a3);
  fe2_add_lazy(sb, b.a2, b.a3);
  norm(sb.c0), norm(sb.c1);
  fe2_mul(u, sa, sb);
  fe2_sub_r(u, u, t2);
  fe2_sub_r(r.c1.c2, u, t3);
}
// a (b0 + b1 v): 5 Fp2 products; a, b0, b1 normalized and < 2.2 p
HD void fe6_mul_01(fe6 &r, const fe6 &a, const fe2 &b0, const fe2 &b1) {
  fe2 t0, t1, s0, s1, c0, c1, c2;
  fe2_mul(t0, a.c0, b0);
  fe2_mul(t1, a.c1, b1);
  fe2_add_lazy(s0, a.c1, a.c2);
  fe2_mul(c0, s0, b1);
  fe2_sub_r(c0, c0, t1);
  fe2_mul_xi_r(c0, c0);
  fe2_add_r(c0, c0, t0);
  fe2_add_lazy(s0, a.c0, a.c1);
  fe2_add_lazy(s1, b0, b1);
  norm(s1.c0), norm(s1.c1);
  fe2_mul(c1, s0, s1);
  fe2_sub_r(c1, c1, t0);
  fe2_sub_r(c1, c1, t1);
  fe2_add_lazy(s0, a.c0, a.c2);
  fe2_mul(c2, s0, b0);
  fe2_sub_r(c2, c2, t0);
  fe2_add_r(c2, c2, t1);
  r.c0 = c0;
  r.c1 = c1;
  r.c2 = c2;
}
// a (b1 v): 3 Fp2 products
HD void fe6_mul_1(fe6 &r, const fe6 &a, const fe2 &b1) {
  fe2 c0, c1, c2;
  fe2_mul(c0, a.c2, b1);
  fe2_mul_xi_r(c0, c0);
  fe2_mul(c1, a.c0, b1);
  fe2_mul(c2, a.c1, b1);
  r.c0 = c0;
  r.c1 = c1;
  r.c2 = c2;
}
// f (l0 + l2 w^2 + l3 w^3) = f ((l0 + l2 v) + (l3 v) w): 13 Fp2 products
HD void fe12_mul_034(fe12 &r, const fe12 &a, const sp &s) {
  fe6 t0, t1, u;
  fe6_mul_01(t0, a.c0, s.a0, s.a2);
  fe6_mul_1(t1, a.c1, s.a3);
  fe6_add(u, a.c0, a.c1);
  fe2 l23;
  fe2_add_lazy(l23, s.a2, s.a3);
  norm(l23.c0), norm(l23.c1);
  fe6_mul_01(u, u, s.a0, l23);
  fe6_sub_r(u, u, t0);
  fe6_sub_r(r.c1, u, t1);
  fe2 x;
  fe2_mul_xi_r(x, t1.c2);  // t1 v
  fe2_add_r(r.c0.c0, t0.c0, x);
  fe2_add_r(r.c0.c1, t0.c1, t1.c0);
  fe2_add_r(r.c0.c2, t0.c2, t1.c1);
}
// fe12_mul_034 with t1 = a.c1 s.a3 parked in a per-lane stash (LDS in k_ml_group28, word i of
// the lane at st[i * stride]) while the Karatsuba middle product runs: 84 fewer live registers
HD void fe6_stash(uint32_t *st, uint32_t stride, const fe6 &a) {
  const uint32_t *w = reinterpret_cast<const uint32_t *>(&a);
#pragma unroll
  for (int i = 0; i < 84; i++) st[i * stride] = w[i];
}
HD void fe6_unstash(fe6 &a, const uint32_t *st, uint32_t stride) {
  uint32_t *w = reinterpret_cast<uint32_t *>(&a);
#pragma unroll
  for (int i = 0; i < 84; i++) w[i] = st[i * stride];
}
// and the first 70 words of t0 at st[(84 + i) * stride] during it (154 words: 4 waves of 64
// lanes per CU stay within 160 KB of LDS)
HD void fe12_mul_034_st(fe12 &r, const fe12 &a, const sp &s, uint32_t *st, uint32_t stride) {
  {
    fe6 t1;
    fe6_mul_1(t1, a.c1, s.a3);
    fe6_stash(st, stride, t1);
  }
  fe6 t0, u;
  fe6_mul_01(t0, a.c0, s.a0, s.a2);
  fe6_add(u, a.c0, a.c1);
  {
    const uint32_t *w = reinterpret_cast<const uint32_t *>(&t0);
#pragma unroll
    for (int i = 0; i < 70; i++) st[(84 + i) * stride] = w[i];
  }
  fe2 l23;
  fe2_add_lazy(l23, s.a2, s.a3);
  norm(l23.c0), norm(l23.c1);
  fe6_mul_01(u, u, s.a0, l23);
  {
    uint32_t *w = reinterpret_cast<uint32_t *>(&t0);
#pragma unroll
    for (int i = 0; i < 70; i++) w[i] = st[(84 + i) * stride];
  }
  fe6_sub_r(u, u, t0);
  fe6 t1;
  fe6_unstash(t1, st, stride);
  fe6_sub_r(r.c1, u, t1);
  fe2 x;
  fe2_mul_xi_r(x, t1.c2);
  fe2_add_r(r.c0.c0, t0.c0, x);
  fe2_add_r(r.c0.c1, t0.c1, t1.c0);
  fe2_add_r(r.c0.c2, t0.c2, t1.c1);
}
// f <- f (a0 + a2 w^2 + a3 w^3) with ONE reduction per output Fp coordinate (lazy reduction):
// in the w basis f = sum f_i w^i (f0 = c0.c0, f1 = c1.c0, f2 = c0.c1, f3 = c1.c1, f4 = c0.c2,
// f5 = c1.c2; w^6 = xi) the product's coefficients are
//   r0 = f0 a0 + f4 b2 + f3 b3      r3 = f3 a0 + f1 a2 + f0 a3
//   r1 = f1 a0 + f5 b2 + f4 b3      r4 = f4 a0 + f2 a2 + f1 a3
//   r2 = f2 a0 + f0 a2 + f5 b3      r5 = f5 a0 + f3 a2 + f2 a3       (b = xi a)
// so each Fp coordinate is six Fp products, summed in one product-scanning pass and reduced
// once (mul6): 72 products + 12 reductions against the Karatsuba form's 52 products + 26
// reductions and ~60 Fp additions/subtractions (the r04 kernel), and no Fp12 temporaries:
// the outputs are written in place in the order r3 r4 r5 r2 r0 r1, which frees each input
// after its last use, with at most three outputs parked.  The minus signs of Re(x y) =
// x0 y0 - x1 y1 ride in negated line operands (4p - y1, limbs < 2^29).  Line coefficients
// normalized and < 1.1 p; f normalized and < 1.1 p; outputs normalized and < 1.02 p.
HD void fe2_mul3_acc(fe2 &r, const fe2 &x, const fe2 &u, const fe &nu1, const fe2 &y, const fe2 &v,
                     const fe &nv1, const fe2 &z, const fe2 &t, const fe &nt1) {
  // r = x u + y v + z t (Fp2), nu1 = 4p - u.c1 etc.
  mul6(r.c0, x.c0, u.c0, x.c1, nu1, y.c0, v.c0, y.c1, nv1, z.c0, t.c0, z.c1, nt1);
  mul6(r.c1, x.c0, u.c1, x.c1, u.c0, y.c0, v.c1, y.c1, v.c0, z.c0, t.c1, z.c1, t.c0);
}
HD void fe12_mul_034_lazy(fe12 &f, const sp &s) {
  fe2 &f0 = f.c0.c0, &f1 = f.c1.c0, &f2 = f.c0.c1, &f3 = f.c1.c1, &f4 = f.c0.c2, &f5 = f.c1.c2;
  fe n0, n2, n3;
  neg_lazy(n0, s.a0.c1);
  neg_lazy(n2, s.a2.c1);
  neg_lazy(n3, s.a3.c1);
  fe2 r3, r4, r5, x;
  fe2_mul3_acc(r3, f3, s.a0, n0, f1, s.a2, n2, f0, s.a3, n3);
  fe2_mul3_acc(r4, f4, s.a0, n0, f2, s.a2, n2, f1, s.a3, n3);
  fe2_mul3_acc(r5, f5, s.a0, n0, f3, s.a2, n2, f2, s.a3, n3);
  fe2 b3, b2;
  sub(b3.c0, s.a3.c0, s.a3.c1);  // xi a3 (< 5.1 p, normalized)
  add(b3.c1, s.a3.c0, s.a3.c1);
  neg_lazy(n3, b3.c1);
  fe2_mul3_acc(x, f2, s.a0, n0, f0, s.a2, n2, f5, b3, n3);
  f2 = x;  // r2 (f2's last use)
  sub(b2.c0, s.a2.c0, s.a2.c1);  // xi a2
  add(b2.c1, s.a2.c0, s.a2.c1);
  neg_lazy(n2, b2.c1);
  fe2_mul3_acc(x, f0, s.a0, n0, f4, b2, n2, f3, b3, n3);
  f0 = x;  // r0 (last use of f0 and f3)
  f3 = r3;
  fe2_mul3_acc(x, f1, s.a0, n0, f5, b2, n2, f4, b3, n3);
  f1 = x;  // r1 (last use of f1, f4, f5)
  f4 = r4;
  f5 = r5;
}

// fe12_mul_034_lazy with the three parked outputs (r3, r4, r5: 84 words) in a per-lane stash
// (LDS in k_ml_group28, word i of the lane at st[i * stride]): 84 fewer live registers
HD void fe2_stash(uint32_t *st, uint32_t stride, const fe2 &a) {
  const uint32_t *w = reinterpret_cast<const uint32_t *>(&a);
#pragma unroll
  for (int i = 0; i < 28; i++) st[i * stride] = w[i];
}
HD void fe2_unstash(fe2 &a, const uint32_t *st, uint32_t stride) {
  uint32_t *w = reinterpret_cast<uint32_t *>(&a);
#pragma unroll
  for (int i = 0; i < 28; i++) w[i] = st[i * stride];
}
HD void fe12_mul_034_lazy_st(fe12 &f, const sp &s, uint32_t *st, uint32_t stride) {
  fe2 &f0 = f.c0.c0, &f1 = f.c1.c0, &f2 = f.c0.c1, &f3 = f.c1.c1, &f4 = f.c0.c2, &f5 = f.c1.c2;
  fe n0, n2, n3;
  neg_lazy(n0, s.a0.c1);
  neg_lazy(n2, s.a2.c1);
  neg_lazy(n3, s.a3.c1);
  fe2 x;
  fe2_mul3_acc(x, f3, s.a0, n0, f1, s.a2, n2, f0, s.a3, n3);
  fe2_stash(st, stride, x);  // r3
  fe2_mul3_acc(x, f4, s.a0, n0, f2, s.a2, n2, f1, s.a3, n3);
  fe2_stash(st + 28 * stride, stride, x);  // r4
  fe2_mul3_acc(x, f5, s.a0, n0, f3, s.a2, n2, f2, s.a3, n3);
  fe2_stash(st + 56 * stride, stride, x);  // r5
  fe2 b3, b2;
  sub(b3.c0, s.a3.c0, s.a3.c1);  // xi a3
  add(b3.c1, s.a3.c0, s.a3.c1);
  neg_lazy(n3, b3.c1);
  fe2_mul3_acc(x, f2, s.a0, n0, f0, s.a2, n2, f5, b3, n3);
  f2 = x;  // r2
  sub(b2.c0, s.a2.c0, s.a2.c1);  // xi a2
  add(b2.c1, s.a2.c0, s.a2.c1);
  neg_lazy(n2, b2.c1);
  fe2_mul3_acc(x, f0, s.a0, n0, f4, b2, n2, f3, b3, n3);
  f0 = x;  // r0
  fe2_unstash(f3, st, stride);
  fe2_mul3_acc(x, f1, s.a0, n0, f5, b2, n2, f4, b3, n3);
  f1 = x;  // r1
  fe2_unstash(f4, st + 28 * stride, stride);
  fe2_unstash(f5, st + 56 * stride, stride);
}

// ---- r06: the same product with Karatsuba Fp2 products (fe2_mul3k: 9 products of 196 terms per
// output Fp2 coordinate instead of 12; tools/gen_fpmul28.py emit_kara3).  Each output r_k (Fp2)
// is x_1 u_1 + x_2 u_2 + x_3 u_3 with x from f and u a line coefficient; the line's limbwise
// sums us = u.c0 + u.c1 are formed once per line, f's inside the product.  Outputs < 1.03 p
// (the c0 coordinate carries a bias of 17 p^2, a multiple of p), normalized.
HD void fe2_sum(fe &r, const fe2 &a) { add_lazy(r, a.c0, a.c1); }  // limbs < 2^29
HD void fe2_mul3k(fe2 &r, const fe2 &x0, const fe2 &u0, const fe &u0s, const fe2 &x1, const fe2 &u1,
                  const fe &u1s, const fe2 &x2, const fe2 &u2, const fe &u2s) {
#if defined(__HIP_DEVICE_COMPILE__)
  fe2_mul3k_dev(r.c0, r.c1, x0.c0, x0.c1, u0.c0, u0.c1, u0s, x1.c0, x1.c1, u1.c0, u1.c1, u1s, x2.c0, x2.c1, u2.c0,
                u2.c1, u2s);
#else
  (void)u0s, (void)u1s, (void)u2s;  // the host computes the same value (mod p) the schoolbook way
  fe n0, n1, n2;
  neg_lazy(n0, u0.c1);
  neg_lazy(n1, u1.c1);
  neg_lazy(n2, u2.c1);
  fe2_mul3_acc(r, x0, u0, n0, x1, u1, n1, x2, u2, n2);
#endif
}
HD void fe12_mul_034_kara_st(fe12 &f, const sp &s, uint32_t *st, uint32_t stride) {
  fe2 &f0 = f.c0.c0, &f1 = f.c1.c0, &f2 = f.c0.c1, &f3 = f.c1.c1, &f4 = f.c0.c2, &f5 = f.c1.c2;
  fe s0, s2, s3;
  fe2_sum(s0, s.a0);
  fe2_sum(s2, s.a2);
  fe2_sum(s3, s.a3);
  fe2 x;
  fe2_mul3k(x, f3, s.a0, s0, f1, s.a2, s2, f0, s.a3, s3);
  fe2_stash(st, stride, x);  // r3
  fe2_mul3k(x, f4, s.a0, s0, f2, s.a2, s2, f1, s.a3, s3);
  fe2_stash(st + 28 * stride, stride, x);  // r4
  fe2_mul3k(x, f5, s.a0, s0, f3, s.a2, s2, f2, s.a3, s3);
  fe2_stash(st + 56 * stride, stride, x);  // r5
  fe2 b3, b2;
  sub(b3.c0, s.a3.c0, s.a3.c1);  // xi a3 (< 5.1 p, normalized)
  add(b3.c1, s.a3.c0, s.a3.c1);
  fe2_sum(s3, b3);
  fe2_mul3k(x, f2, s.a0, s0, f0, s.a2, s2, f5, b3, s3);
  f2 = x;  // r2
  sub(b2.c0, s.a2.c0, s.a2.c1);  // xi a2
  add(b2.c1, s.a2.c0, s.a2.c1);
  fe2_sum(s2, b2);
  fe2_mul3k(x, f0, s.a0, s0, f4, b2, s2, f3, b3, s3);
  f0 = x;  // r0
  fe2_unstash(f3, st, stride);
  fe2_mul3k(x, f1, s.a0, s0, f5, b2, s2, f4, b3, s3);
  f1 = x;  // r1
  fe2_unstash(f4, st + 28 * stride, stride);
  fe2_unstash(f5, st + 56 * stride, stride);
}

// (a0 + a2 w^2 + a3 w^3)(b0 + b2 w^2 + b3 w^3) with one reduction per output Fp coordinate:
//   r0 = a0 b0 + a3 (xi b3), r1 = 0, r2 = a0 b2 + a2 b0, r3 = a0 b3 + a3 b0, r4 = a2 b2,
//   r5 = a2 b3 + a3 b2
// (four products per coordinate, two for r4).  Inputs normalized, < 1.1 p; outputs < 1.01 p.
HD void sp_mul_sp_lazy(fe12 &r, const sp &a, const sp &b) {
  fe n0, n2, n3;
  neg_lazy(n0, b.a0.c1);
  neg_lazy(n2, b.a2.c1);
  neg_lazy(n3, b.a3.c1);
  // x u + y v (Fp2), nu1 = 4p - u.c1
  auto mul2_acc = [](fe2 &o, const fe2 &x, const fe2 &u, const fe &nu1, const fe2 &y, const fe2 &v,
                     const fe &nv1) {
    mul4(o.c0, x.c0, u.c0, x.c1, nu1, y.c0, v.c0, y.c1, nv1);
    mul4(o.c1, x.c0, u.c1, x.c1, u.c0, y.c0, v.c1, y.c1, v.c0);
  };
  mul2_acc(r.c0.c1, a.a0, b.a2, n2, a.a2, b.a0, n0);                   // r2
  mul2_acc(r.c1.c1, a.a0, b.a3, n3, a.a3, b.a0, n0);                   // r3
  mul2_acc(r.c1.c2, a.a2, b.a3, n3, a.a3, b.a2, n2);                   // r5
  mul2(r.c0.c2.c0, a.a2.c0, b.a2.c0, a.a2.c1, n2);                     // r4
  mul2(r.c0.c2.c1, a.a2.c0, b.a2.c1, a.a2.c1, b.a2.c0);
  fe2 x;
  sub(x.c0, b.a3.c0, b.a3.c1);  // xi b3
  add(x.c1, b.a3.c0, b.a3.c1);
  neg_lazy(n3, x.c1);
  mul2_acc(r.c0.c0, a.a0, b.a0, n0, a.a3, x, n3);                      // r0
  fe2_zero(r.c1.c0);                                                   // r1
}

// sparse line from engine-form line coefficients and an engine-form g1s point, with no
// conversion: the product of two engine-form words over R = 2^392 is the radix-2^28 form of
// L P times 2^-16, a scalar that the final exponentiation removes (as the g1s scaling does)
HD void sp_from_engine(sp &s, const fp2 &L0, const fp2 &L2, const fp2 &L3, const fp &Px,
                       const fp &Py, const fp &Pc) {
  fe q, t;
  repack_in(q, Pc);
  repack_in(t, L0.c0), mul(s.a0.c0, t, q);
  repack_in(t, L0.c1), mul(s.a0.c1, t, q);
  repack_in(q, Px);
  repack_in(t, L2.c0), mul(s.a2.c0, t, q);
  repack_in(t, L2.c1), mul(s.a2.c1, t, q);
  repack_in(q, Py);
  repack_in(t, L3.c0), mul(s.a3.c0, t, q);
  repack_in(t, L3.c1), mul(s.a3.c1, t, q);
}
HD void sp_identity(sp &s) {  // 2^-392 (raw limb 1): a nonzero scalar
  fe2_zero(s.a0);
  s.a0.c0.l[0] = 1;
  fe2_zero(s.a2);
  fe2_zero(s.a3);
}
HD void sp_to_fe12(fe12 &r, const sp &s) {
  r.c0.c0 = s.a0;
  r.c0.c1 = s.a2;
  fe2_zero(r.c0.c2);
  fe2_zero(r.c1.c0);
  r.c1.c1 = s.a3;
  fe2_zero(r.c1.c2);
}
// engine-form words of the value (canonical): f times 2^8 in the engine's reading
HD void fe12_to_engine_scaled(fp12 &r, const fe12 &a) {
  const fe *src[12] = {&a.c0.c0.c0, &a.c0.c0.c1, &a.c0.c1.c0, &a.c0.c1.c1, &a.c0.c2.c0, &a.c0.c2.c1,
                       &a.c1.c0.c0, &a.c1.c0.c1, &a.c1.c1.c0, &a.c1.c1.c1, &a.c1.c2.c0, &a.c1.c2.c1};
  fp *dst[12] = {&r.c0.c0.c0, &r.c0.c0.c1, &r.c0.c1.c0, &r.c0.c1.c1, &r.c0.c2.c0, &r.c0.c2.c1,
                 &r.c1.c0.c0, &r.c1.c0.c1, &r.c1.c1.c0, &r.c1.c1.c1, &r.c1.c2.c0, &r.c1.c2.c1};
#pragma unroll
  for (int i = 0; i < 12; i++) {
    fe t = *src[i];
    (void)sub_p_if_geq(t);  // < 1.1 p -> < p
    repack_out(*dst[i], t);
  }
}

}  // namespace r28
}  // namespace gbls
