// Row-distributed Fp12 engine for the latency regime: the wave12 engine's three-level
// Karatsuba Fp12 product (54 Fp products, bls_wave12.h) with every Fp product on its own
// 16-lane row in the row-distributed field layer (bls_dfp.h), so that one Fp12 product costs
// one row product (~0.46 us on MI355X, against ~1.2 us for a one-lane product) plus two
// lane-local recombination rounds (the POST1 / POST2 rounds composed into one) -- the serial
// Fp12 chains of one segment (Horner over the Miller events, the final exponentiation) run
// ~4x faster.  One workgroup of W12D_THREADS (56 rows) per chain; images live in LDS as
// 12 slots of 16 words (coefficient c at words [16 c, 16 c + 16), lane j's limb at word j).
//
// Value contract: products < 1.0001 p; R1 values < 14.001 p; Fp12 coefficients (R2
// outputs, conj, Frobenius) < 128 p; a presum of <= 8 coefficients < 1024 p < 2^392, the
// product's input bound.  Every stored limb is < 2^28 + 2^9.
#pragma once
#include "bls_dfp.h"

namespace gbls {
namespace w12d {

constexpr int ROWS = 56;
constexpr int THREADS = ROWS * 16;  // 14 waves
constexpr int IMG = 12 * 16;        // words per Fp12 image
constexpr int WS = dfp::W12D_NSLOT * 16;

struct Eng {
  dfp::Tabs t;
  uint32_t row, j;
  uint32_t pre[2], r1[3], r2[2];  // packed plan bytes of this row (product)
  uint32_t sl[2], srp, srn, s1[3], s2[2];  // ... and of the squaring
  uint32_t *ws;                   // WS words of LDS
};

__device__ __forceinline__ uint32_t byte_of(const uint32_t *w, int k) { return (w[k >> 2] >> (8 * (k & 3))) & 0xffu; }

// every thread of the workgroup; ws = WS words of LDS
__device__ __forceinline__ void begin(Eng &e, uint32_t *ws) {
  dfp::load_tabs(e.t);
  e.row = threadIdx.x >> 4;
  e.j = threadIdx.x & 15;
  e.ws = ws;
  const uint32_t r = e.row;
  uint32_t b[12];
#pragma unroll
  for (int k = 0; k < 8; k++) b[k] = r < 54 ? dfp::W12D_PRE[r][k] : 12u;
  e.pre[0] = b[0] | b[1] << 8 | b[2] << 16 | b[3] << 24;
  e.pre[1] = b[4] | b[5] << 8 | b[6] << 16 | b[7] << 24;
#pragma unroll
  for (int k = 0; k < 12; k++) b[k] = r < 18 ? dfp::W12D_R1[r][k] : (uint32_t)dfp::W12D_ZERO;
  e.r1[0] = b[0] | b[1] << 8 | b[2] << 16 | b[3] << 24;
  e.r1[1] = b[4] | b[5] << 8 | b[6] << 16 | b[7] << 24;
  e.r1[2] = b[8] | b[9] << 8 | b[10] << 16 | b[11] << 24;
#pragma unroll
  for (int k = 0; k < 5; k++) b[k] = r < 12 ? dfp::W12D_R2[r][k] : (uint32_t)dfp::W12D_ZERO;
  e.r2[0] = b[0] | b[1] << 8 | b[2] << 16 | b[3] << 24;
  e.r2[1] = b[4];
  // squaring plan (36 product rows)
#pragma unroll
  for (int k = 0; k < 8; k++) b[k] = r < 36 ? dfp::W12S_L[r][k] : 12u;
  e.sl[0] = b[0] | b[1] << 8 | b[2] << 16 | b[3] << 24;
  e.sl[1] = b[4] | b[5] << 8 | b[6] << 16 | b[7] << 24;
#pragma unroll
  for (int k = 0; k < 4; k++) b[k] = r < 36 ? dfp::W12S_RP[r][k] : 12u;
  e.srp = b[0] | b[1] << 8 | b[2] << 16 | b[3] << 24;
#pragma unroll
  for (int k = 0; k < 4; k++) b[k] = r < 36 ? dfp::W12S_RN[r][k] : 12u;
  e.srn = b[0] | b[1] << 8 | b[2] << 16 | b[3] << 24;
#pragma unroll
  for (int k = 0; k < 12; k++) b[k] = r < 18 ? dfp::W12S_R1[r][k] : (uint32_t)dfp::W12D_ZERO;
  e.s1[0] = b[0] | b[1] << 8 | b[2] << 16 | b[3] << 24;
  e.s1[1] = b[4] | b[5] << 8 | b[6] << 16 | b[7] << 24;
  e.s1[2] = b[8] | b[9] << 8 | b[10] << 16 | b[11] << 24;
#pragma unroll
  for (int k = 0; k < 5; k++) b[k] = r < 12 ? dfp::W12S_R2[r][k] : (uint32_t)dfp::W12D_ZERO;
  e.s2[0] = b[0] | b[1] << 8 | b[2] << 16 | b[3] << 24;
  e.s2[1] = b[4];
  if (threadIdx.x < 16) ws[16 * dfp::W12D_ZERO + threadIdx.x] = 0;
  __syncthreads();
}

// sum of the row's <= 8 planned coefficients of image a (index 12 = the zero slot)
__device__ __forceinline__ uint32_t presum(const Eng &e, const uint32_t *a) {
  uint32_t s = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) {
    const uint32_t c = byte_of(e.pre, k);
    const uint32_t *src = c == 12 ? e.ws + 16 * dfp::W12D_ZERO : a + 16 * c;
    s += src[e.j];
  }
  return dfp::norm(s);  // limbs < 8 (2^28 + 2^9) -> < 2^28 + 8
}

// c = a b (c may alias a or b).  All threads call it.
__device__ __forceinline__ void mul(Eng &e, uint32_t *c, const uint32_t *a, const uint32_t *b) {
  if (e.row < 54) {
    const uint32_t x = presum(e, a);
    const uint32_t y = a == b ? x : presum(e, b);
    const uint32_t p = dfp::mul(x, y, e.t);
    e.ws[16 * e.row + e.j] = p;
  }
  __syncthreads();
  if (e.row < 18) {  // R1: 8p + (<= 6 products) - (<= 6 products)
    uint32_t s = dfp::konst(dfp::K_BIAS_R1);
#pragma unroll
    for (int k = 0; k < 6; k++) s += e.ws[16 * byte_of(e.r1, k) + e.j];
#pragma unroll
    for (int k = 6; k < 12; k++) s -= e.ws[16 * byte_of(e.r1, k) + e.j];
    e.ws[16 * (54 + e.row) + e.j] = dfp::norm(s);
  }
  __syncthreads();
  if (e.row < 12) {  // R2: 32p + (<= 3 R1 values) - (<= 2 R1 values)
    uint32_t s = dfp::konst(dfp::K_BIAS_R2);
#pragma unroll
    for (int k = 0; k < 3; k++) s += e.ws[16 * byte_of(e.r2, k) + e.j];
#pragma unroll
    for (int k = 3; k < 5; k++) s -= e.ws[16 * byte_of(e.r2, k) + e.j];
    c[16 * e.row + e.j] = dfp::norm(s);
  }
  __syncthreads();
}

// c = a^2 (c may alias a): 36 row products (the three-level Karatsuba tree with Fp2
// squarings (x0 + x1)(x0 - x1), x0 x1 at the leaves, tools/gen_wave12.py build_sqr), then the
// product's R1 / R2 rounds with the squaring's plan.  All threads call it.
__device__ __forceinline__ void sqr(Eng &e, uint32_t *c, const uint32_t *a) {
  if (e.row < 36) {
    const uint32_t *zero = e.ws + 16 * dfp::W12D_ZERO;
    uint32_t x = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const uint32_t q = byte_of(e.sl, k);
      x += (q == 12 ? zero : a + 16 * q)[e.j];
    }
    uint32_t y = dfp::konst(dfp::K_BIAS_SQ);
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const uint32_t q = (e.srp >> (8 * k)) & 0xffu;
      y += (q == 12 ? zero : a + 16 * q)[e.j];
    }
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const uint32_t q = (e.srn >> (8 * k)) & 0xffu;
      y -= (q == 12 ? zero : a + 16 * q)[e.j];
    }
    // x: <= 8 coefficients (< 1024 p); y: 1024 p + <= 4 - <= 4 coefficients (< 1536 p)
    const uint32_t p = dfp::mul(dfp::norm(x), dfp::norm(y), e.t);
    e.ws[16 * e.row + e.j] = p;
  }
  __syncthreads();
  if (e.row < 18) {
    uint32_t s = dfp::konst(dfp::K_BIAS_R1);
#pragma unroll
    for (int k = 0; k < 6; k++) s += e.ws[16 * byte_of(e.s1, k) + e.j];
#pragma unroll
    for (int k = 6; k < 12; k++) s -= e.ws[16 * byte_of(e.s1, k) + e.j];
    e.ws[16 * (54 + e.row) + e.j] = dfp::norm(s);
  }
  __syncthreads();
  if (e.row < 12) {
    uint32_t s = dfp::konst(dfp::K_BIAS_R2);
#pragma unroll
    for (int k = 0; k < 3; k++) s += e.ws[16 * byte_of(e.s2, k) + e.j];
#pragma unroll
    for (int k = 3; k < 5; k++) s -= e.ws[16 * byte_of(e.s2, k) + e.j];
    c[16 * e.row + e.j] = dfp::norm(s);
  }
  __syncthreads();
}

// c = conj(a) = a^(p^6): the w-odd half (coefficients 6..11) negated
__device__ __forceinline__ void conj(Eng &e, uint32_t *c, const uint32_t *a) {
  if (e.row < 12) {
    const uint32_t x = a[16 * e.row + e.j];
    c[16 * e.row + e.j] = e.row < 6 ? x : dfp::sub(0, x, dfp::K_BIAS_NEG);
  }
  __syncthreads();
}
__device__ __forceinline__ void copy(Eng &e, uint32_t *c, const uint32_t *a) {
  if (e.row < 12) c[16 * e.row + e.j] = a[16 * e.row + e.j];
  __syncthreads();
}
// Frobenius: the Fp2 coefficient of w^f (f = 2 jj + h) -> conj(x) gamma1_f.  Row r < 12 makes
// component r & 1 of Fp2 coefficient q = r >> 1 (h = q & 1, jj = q >> 1): one dual product.
// c must not alias a.
__device__ __forceinline__ void frob(Eng &e, uint32_t *c, const uint32_t *a) {
  if (e.row < 12) {
    const uint32_t q = e.row >> 1, k = e.row & 1, h = q & 1, jj = q >> 1, f = 2 * jj + h;
    const uint32_t ci = h * 6 + jj * 2;
    const uint32_t x0 = a[16 * ci + e.j], x1 = a[16 * (ci + 1) + e.j];
    const uint32_t g0 = dfp::K_FROB1[f][0][e.j], g1 = dfp::K_FROB1[f][1][e.j];
    const uint32_t nx1 = dfp::sub(0, x1, dfp::K_BIAS_NEG);
    // (x0 - x1 u)(g0 + g1 u) = (x0 g0 + x1 g1) + (x0 g1 - x1 g0) u
    const uint32_t r = k == 0 ? dfp::mul2(x0, g0, x1, g1, e.t) : dfp::mul2(x0, g1, nx1, g0, e.t);
    c[16 * (ci + k) + e.j] = r;
  }
  __syncthreads();
}
// Frobenius^2: coefficient (h, jj, k) of w^f times the Fp constant gamma2_f (f = 2 jj + h)
__device__ __forceinline__ void frob2(Eng &e, uint32_t *c, const uint32_t *a) {
  if (e.row < 12) {
    const uint32_t h = e.row / 6, jj = (e.row % 6) >> 1, f = 2 * jj + h;
    c[16 * e.row + e.j] = dfp::mul(a[16 * e.row + e.j], dfp::K_FROB2[f][e.j], e.t);
  }
  __syncthreads();
}
// c = a^x (x = -|x|): a^|x| by square-and-multiply, then conj (a^x on the cyclotomic
// subgroup; the verdict's chain uses it as the fixed exponentiation Psi).  c must not alias a.
__device__ __forceinline__ void exp_x(Eng &e, uint32_t *c, const uint32_t *a) {
  copy(e, c, a);
  for (int i = 62; i >= 0; i--) {
    sqr(e, c, c);
    if ((dfp::X_ABS >> i) & 1) mul(e, c, c, a);
  }
  conj(e, c, c);
}
// image <- engine-form Fp12 words (12 coefficients x 12 words) as repacked limbs: the value
// times the Fp scalar 2^-64 (harmless for Miller values, whose final exponentiation kills
// every Fp* factor)
__device__ __forceinline__ void load_scaled(Eng &e, uint32_t *c, const uint32_t *words) {
  if (e.row < 12) c[16 * e.row + e.j] = dfp::from_words_scaled(words + 12 * e.row);
  __syncthreads();
}
// engine-form canonical words of image a (12 coefficients x 12 words)
__device__ __forceinline__ void store_words(Eng &e, uint32_t *words, const uint32_t *a) {
  if (e.row < 12) dfp::to_words(words + 12 * e.row, a[16 * e.row + e.j], e.t);
}
// flags[r] = coefficient r of image a is 0 mod p, for r in [lo, hi); then a barrier
__device__ __forceinline__ void zero_flags(Eng &e, int *flags, const uint32_t *a, uint32_t lo,
                                           uint32_t hi) {
  if (e.row >= lo && e.row < hi) {
    const bool z = dfp::is_zero(a[16 * e.row + e.j], e.t);
    if (e.j == 0) flags[e.row] = z ? 1 : 0;
  }
  __syncthreads();
}

}  // namespace w12d
}  // namespace gbls
