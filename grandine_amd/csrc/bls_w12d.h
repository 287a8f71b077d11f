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
#include "bls_inv.h"

namespace gbls {
namespace w12d {

constexpr int ROWS = 56;
constexpr int THREADS = ROWS * 16;  // 14 waves
constexpr int IMG = 12 * 16;        // words per Fp12 image
// LDS workspace: the value slots, then every row's packed plan words (kept in LDS rather than
// in registers: with 896 threads a lane has 128 VGPRs, and plan words held across the
// exponentiation chains were spilled to scratch), then the cyclotomic squaring's constants
constexpr int PLAN = dfp::W12D_NSLOT * 16;
constexpr int PW = 20;  // plan words per row
enum : int { P_PRE = 0, P_R1 = 2, P_R2 = 5, P_SL = 7, P_SRP = 9, P_SRN = 10, P_S1 = 11, P_S2 = 14, P_G = 16, P_GC = 18 };
constexpr int GSK = PLAN + ROWS * PW;
constexpr int WS = GSK + 5 * 16;

struct Eng {
  dfp::Tabs t;
  uint32_t row, j;
  uint32_t *ws;        // WS words of LDS
  const uint32_t *pl;  // this row's plan words (ws + PLAN + PW row)
};

// The cyclotomic squaring's product row on physical row r, or -1.  Waves go to the 4 SIMDs
// round-robin (wave w on SIMD w mod 4): GS rows 0..11 (dual products) fill waves 0..2, the
// single products 12..15 wave 3 and 16..17 wave 7, so SIMD 0..2 each run one wave of dual
// products and SIMD 3 two waves of single ones (rows 16..17 on wave 4 put a dual and a single
// wave on SIMD 0: 2.6 single-product times against 2 here).
__device__ __forceinline__ int gs_row(uint32_t r) { return r < 16 ? (int)r : (r == 28 || r == 29) ? (int)r - 12 : -1; }

__device__ __forceinline__ uint32_t byte_of(const uint32_t *w, int k) { return (w[k >> 2] >> (8 * (k & 3))) & 0xffu; }

// every thread of the workgroup; ws = WS words of LDS
__device__ __forceinline__ void begin(Eng &e, uint32_t *ws) {
  dfp::load_tabs(e.t);
  e.row = threadIdx.x >> 4;
  e.j = threadIdx.x & 15;
  e.ws = ws;
  e.pl = ws + PLAN + PW * e.row;
  const uint32_t r = e.row;
  uint32_t b[12], w[PW];
#pragma unroll
  for (int k = 0; k < 8; k++) b[k] = r < 54 ? dfp::W12D_PRE[r][k] : 12u;
  w[P_PRE + 0] = b[0] | b[1] << 8 | b[2] << 16 | b[3] << 24;
  w[P_PRE + 1] = b[4] | b[5] << 8 | b[6] << 16 | b[7] << 24;
#pragma unroll
  for (int k = 0; k < 12; k++) b[k] = r < 18 ? dfp::W12D_R1[r][k] : (uint32_t)dfp::W12D_ZERO;
  w[P_R1 + 0] = b[0] | b[1] << 8 | b[2] << 16 | b[3] << 24;
  w[P_R1 + 1] = b[4] | b[5] << 8 | b[6] << 16 | b[7] << 24;
  w[P_R1 + 2] = b[8] | b[9] << 8 | b[10] << 16 | b[11] << 24;
#pragma unroll
  for (int k = 0; k < 5; k++) b[k] = r < 12 ? dfp::W12D_R2[r][k] : (uint32_t)dfp::W12D_ZERO;
  w[P_R2 + 0] = b[0] | b[1] << 8 | b[2] << 16 | b[3] << 24;
  w[P_R2 + 1] = b[4];
  // squaring plan (36 product rows)
#pragma unroll
  for (int k = 0; k < 8; k++) b[k] = r < 36 ? dfp::W12S_L[r][k] : 12u;
  w[P_SL + 0] = b[0] | b[1] << 8 | b[2] << 16 | b[3] << 24;
  w[P_SL + 1] = b[4] | b[5] << 8 | b[6] << 16 | b[7] << 24;
#pragma unroll
  for (int k = 0; k < 4; k++) b[k] = r < 36 ? dfp::W12S_RP[r][k] : 12u;
  w[P_SRP] = b[0] | b[1] << 8 | b[2] << 16 | b[3] << 24;
#pragma unroll
  for (int k = 0; k < 4; k++) b[k] = r < 36 ? dfp::W12S_RN[r][k] : 12u;
  w[P_SRN] = b[0] | b[1] << 8 | b[2] << 16 | b[3] << 24;
#pragma unroll
  for (int k = 0; k < 12; k++) b[k] = r < 18 ? dfp::W12S_R1[r][k] : (uint32_t)dfp::W12D_ZERO;
  w[P_S1 + 0] = b[0] | b[1] << 8 | b[2] << 16 | b[3] << 24;
  w[P_S1 + 1] = b[4] | b[5] << 8 | b[6] << 16 | b[7] << 24;
  w[P_S1 + 2] = b[8] | b[9] << 8 | b[10] << 16 | b[11] << 24;
#pragma unroll
  for (int k = 0; k < 5; k++) b[k] = r < 12 ? dfp::W12S_R2[r][k] : (uint32_t)dfp::W12D_ZERO;
  w[P_S2 + 0] = b[0] | b[1] << 8 | b[2] << 16 | b[3] << 24;
  w[P_S2 + 1] = b[4];
  // cyclotomic squaring plan (18 product rows, 12 combine rows)
  const int gr = gs_row(r);
  w[P_G + 0] = gr >= 0 ? dfp::W12G_ROW[gr][0] : 0xccccccccu;
  w[P_G + 1] = gr >= 0 ? dfp::W12G_ROW[gr][1] : 0x01cccccu;
  w[P_GC + 0] = r < 12 ? dfp::W12G_COMB[r][0] : 0x48484848u;
  w[P_GC + 1] = r < 12 ? dfp::W12G_COMB[r][1] : 0x48484848u;
  if (e.j == 0) {
#pragma unroll
    for (int k = 0; k < PW; k++) ws[PLAN + PW * r + k] = w[k];
  }
  if (threadIdx.x < 80) ws[GSK + threadIdx.x] = dfp::K_GS[threadIdx.x >> 4][threadIdx.x & 15];
  if (threadIdx.x < 16) ws[16 * dfp::W12D_ZERO + threadIdx.x] = 0;
  __syncthreads();
}

// sum of the row's <= 8 planned coefficients of image a (index 12 = the zero slot)
__device__ __forceinline__ uint32_t presum(const Eng &e, const uint32_t *a) {
  uint32_t s = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) {
    const uint32_t c = byte_of(e.pl + P_PRE, k);
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
    for (int k = 0; k < 6; k++) s += e.ws[16 * byte_of(e.pl + P_R1, k) + e.j];
#pragma unroll
    for (int k = 6; k < 12; k++) s -= e.ws[16 * byte_of(e.pl + P_R1, k) + e.j];
    e.ws[16 * (54 + e.row) + e.j] = dfp::norm(s);
  }
  __syncthreads();
  if (e.row < 12) {  // R2: 32p + (<= 3 R1 values) - (<= 2 R1 values)
    uint32_t s = dfp::konst(dfp::K_BIAS_R2);
#pragma unroll
    for (int k = 0; k < 3; k++) s += e.ws[16 * byte_of(e.pl + P_R2, k) + e.j];
#pragma unroll
    for (int k = 3; k < 5; k++) s -= e.ws[16 * byte_of(e.pl + P_R2, k) + e.j];
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
      const uint32_t q = byte_of(e.pl + P_SL, k);
      x += (q == 12 ? zero : a + 16 * q)[e.j];
    }
    uint32_t y = dfp::konst(dfp::K_BIAS_SQ);
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const uint32_t q = (e.pl[P_SRP] >> (8 * k)) & 0xffu;
      y += (q == 12 ? zero : a + 16 * q)[e.j];
    }
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const uint32_t q = (e.pl[P_SRN] >> (8 * k)) & 0xffu;
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
    for (int k = 0; k < 6; k++) s += e.ws[16 * byte_of(e.pl + P_S1, k) + e.j];
#pragma unroll
    for (int k = 6; k < 12; k++) s -= e.ws[16 * byte_of(e.pl + P_S1, k) + e.j];
    e.ws[16 * (54 + e.row) + e.j] = dfp::norm(s);
  }
  __syncthreads();
  if (e.row < 12) {
    uint32_t s = dfp::konst(dfp::K_BIAS_R2);
#pragma unroll
    for (int k = 0; k < 3; k++) s += e.ws[16 * byte_of(e.pl + P_S2, k) + e.j];
#pragma unroll
    for (int k = 3; k < 5; k++) s -= e.ws[16 * byte_of(e.pl + P_S2, k) + e.j];
    c[16 * e.row + e.j] = dfp::norm(s);
  }
  __syncthreads();
}

// c = a^2 for a in the cyclotomic subgroup (a^(p^6 + 1) = 1; c may alias a): Granger-Scott,
// 18 row products (12 of them dual, a product plus a constant multiple of an input
// coefficient, so that the squaring's -2 z / +2 z terms ride in the products) and ONE
// combine round, against 36 products and two rounds for sqr.  Plan: tools/gen_dfp.py gs_plan
// (checked there against Fp12 squaring).  Operands: X <= 4 coefficients (< 512 p), Y =
// 512 p + <= 2 - <= 2 coefficients (< 768 p), S = 1024 p + <= 2 - <= 3 coefficients
// (< 1280 p < 2^392); outputs 3 (8 p + <= 5 - <= 6 products) < 40 p.  All threads call it.
__device__ __forceinline__ void cyc_sqr(Eng &e, uint32_t *c, const uint32_t *a) {
  const int gr = gs_row(e.row);
  if (gr >= 0) {
    const uint32_t *zero = e.ws + 16 * dfp::W12D_ZERO;
    const uint32_t w0 = e.pl[P_G], w1 = e.pl[P_G + 1], j = e.j;
    auto co = [&](uint32_t q) { return (q == 12 ? zero : a + 16 * q)[j]; };
    const uint32_t x = co(w0 & 15u) + co((w0 >> 4) & 15u) + co((w0 >> 8) & 15u) + co((w0 >> 12) & 15u);
    uint32_t y = ((w1 >> 20) & 1u) ? dfp::konst(dfp::K_BIAS_GY) : 0u;
    y += co((w0 >> 16) & 15u) + co((w0 >> 20) & 15u);
    y -= co((w0 >> 24) & 15u) + co(w0 >> 28);
    uint32_t p;
    if (((w1 >> 22) & 7u) == 7u) {
      p = dfp::mul(dfp::norm(x), dfp::norm(y), e.t);
    } else {
      uint32_t z = ((w1 >> 21) & 1u) ? dfp::konst(dfp::K_BIAS_GS) : 0u;
      z += co(w1 & 15u) + co((w1 >> 4) & 15u);
      z -= co((w1 >> 8) & 15u) + co((w1 >> 12) & 15u) + co((w1 >> 16) & 15u);
      p = dfp::mul2(dfp::norm(x), dfp::norm(y), dfp::norm(z), e.ws[GSK + 16 * ((w1 >> 22) & 7u) + j], e.t);
    }
    e.ws[16 * gr + j] = p;
  }
  __syncthreads();
  if (e.row < 12) {
    uint32_t pos = 0, neg = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const uint32_t b = byte_of(e.pl + P_GC, k), v = e.ws[16 * (b & 127u) + e.j];
      pos += (b & 128u) ? v << 1 : v;
    }
#pragma unroll
    for (int k = 4; k < 8; k++) {
      const uint32_t b = byte_of(e.pl + P_GC, k), v = e.ws[16 * (b & 127u) + e.j];
      neg += (b & 128u) ? v << 1 : v;
    }
    const uint32_t s = dfp::norm(dfp::konst(dfp::K_BIAS_R1) + pos - neg);
    c[16 * e.row + e.j] = dfp::norm(3u * s);
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
// the same on the cyclotomic subgroup, with cyc_sqr
__device__ __forceinline__ void exp_x_cyc(Eng &e, uint32_t *c, const uint32_t *a) {
  copy(e, c, a);
  for (int i = 62; i >= 0; i--) {
#if defined(GBLS_FEXP_GENERIC_SQR)  // timing experiment
    sqr(e, c, c);
#else
    cyc_sqr(e, c, c);
#endif
#if defined(GBLS_FEXP_DOUBLE_SQR)  // timing experiment
    cyc_sqr(e, c, c);
#endif
    if ((dfp::X_ABS >> i) & 1) mul(e, c, c, a);
  }
  conj(e, c, c);
}

// ---- one Fp inversion by one wave: bls_inv.h's safegcd with the 13 signed 30-bit limbs of
// d, e, f, g spread over lanes 0..12 (lanes 13..63 hold zeros).  The 30 divsteps of a batch
// run on lane 0's limbs as uniform (scalar) values; the matrix updates are one 64-bit
// multiply-add per lane and value, with the division by 2^30 as a one-lane shift (DPP) and
// ONE carry pass: limbs stay redundant (0..12: [-32, 2^30 + 32)), which the divsteps (low 30
// bits of limb 0) and the sign tests (top limb, exact up to values of 2^335, far inside the
// (-2p, p) range argument) tolerate.  The exit test normalizes g fully, only when its low 30
// bits are 0 (at the end, or with probability 2^-30).  26-28 batches for a random input
// (tools/inv_wave_model.py: the same limb arithmetic in Python, checked on 3000 inputs);
// x, out: 12 canonical words in LDS (x = 0 gives garbage, never a hang).  All 64 lanes of
// one wave call it.
__device__ __forceinline__ int32_t inv_lane_shift_dn(int64_t t, int32_t &carry_out) {
  // new limb j = (t_(j+1) & M30) + (t_j >> 30), then one carry pass; top limb signed
  const uint32_t j = threadIdx.x & 63u;
  const int32_t lo = (int32_t)(t & binv::M30);
  const int32_t lo_next = (int32_t)dfp::shl<1>((uint32_t)lo);
  const int64_t n = (int64_t)lo_next + (t >> 30);
  const int32_t c = (int32_t)(n >> 30);
  carry_out = c;
  const int32_t c_in = (int32_t)dfp::shr<1>((uint32_t)c);
  if (j >= (uint32_t)binv::NL) return 0;  // lane 12's carry is not a limb
  return (j < binv::NL - 1 ? (int32_t)(n & binv::M30) : (int32_t)n) + c_in;
}
__device__ __forceinline__ int32_t inv_normalize_full(int32_t x) {  // 12 carry ripples
  const uint32_t j = threadIdx.x & 63u;
#pragma unroll
  for (int k = 0; k < binv::NL - 1; k++) {
    const int32_t c = j < binv::NL - 1 ? (x >> 30) : 0;
    x = (j < binv::NL - 1 ? (x & binv::M30) : x) + (int32_t)dfp::shr<1>((uint32_t)c);
  }
  return x;
}
__device__ __forceinline__ void inv_wave(uint32_t *out, const uint32_t *x) {
  using namespace binv;
  const uint32_t j = threadIdx.x & 63u;
  S30 Pc;
  p30(Pc);
  int32_t pj = 0;
#pragma unroll
  for (int i = 0; i < NL; i++) pj = j == (uint32_t)i ? Pc.v[i] : pj;
  const uint32_t pinv30 = inv32((uint32_t)Pc.v[0]) & (uint32_t)M30;
  int32_t f = pj, g = 0, d = 0, e = j == 0 ? 1 : 0;
  if (j < (uint32_t)NL) {
    const uint32_t bit = 30 * j, w = bit >> 5, sh = bit & 31;
    uint64_t pair = x[w];
    if (w + 1 < 12) pair |= (uint64_t)x[w + 1] << 32;
    g = (int32_t)((pair >> sh) & (uint64_t)M30);
  }
  int32_t eta = -1;
  for (int guard = 0; guard < 40; guard++) {
    const uint32_t f0 = (uint32_t)__builtin_amdgcn_readlane(f, 0);
    const uint32_t g0 = (uint32_t)__builtin_amdgcn_readlane(g, 0);
    Mat t;
    eta = divsteps30(eta, f0, g0, t);
    const int32_t d0 = __builtin_amdgcn_readlane(d, 0), e0 = __builtin_amdgcn_readlane(e, 0);
    const int32_t sd = __builtin_amdgcn_readlane(d, NL - 1) >> 31;
    const int32_t se = __builtin_amdgcn_readlane(e, NL - 1) >> 31;
    int32_t md = (t.u & sd) + (t.v & se), me = (t.q & sd) + (t.r & se);
    const int64_t cd = (int64_t)t.u * d0 + (int64_t)t.v * e0;
    const int64_t ce = (int64_t)t.q * d0 + (int64_t)t.r * e0;
    md -= (int32_t)((pinv30 * (uint32_t)cd + (uint32_t)md) & (uint32_t)M30);
    me -= (int32_t)((pinv30 * (uint32_t)ce + (uint32_t)me) & (uint32_t)M30);
    const int64_t td = (int64_t)t.u * d + (int64_t)t.v * e + (int64_t)pj * md;
    const int64_t te = (int64_t)t.q * d + (int64_t)t.r * e + (int64_t)pj * me;
    const int64_t tf = (int64_t)t.u * f + (int64_t)t.v * g;
    const int64_t tg = (int64_t)t.q * f + (int64_t)t.r * g;
    int32_t c;
    d = inv_lane_shift_dn(td, c);
    e = inv_lane_shift_dn(te, c);
    f = inv_lane_shift_dn(tf, c);
    g = inv_lane_shift_dn(tg, c);
    if ((__builtin_amdgcn_readlane(g, 0) & M30) == 0) {  // g = 0 mod 2^30: test g = 0 exactly
      g = inv_normalize_full(g);
      if (__ballot(g != 0) == 0) break;
    }
  }
  // f = +-1: the sign from its low bits; d = +-x^-1 in (-2p, p), redundant -> canonical words
  const int32_t fsign = (__builtin_amdgcn_readlane(f, 0) & M30) == 1 ? 0 : -1;
  d = inv_normalize_full(d);
  S30 dd;
#pragma unroll
  for (int i = 0; i < NL; i++) dd.v[i] = __builtin_amdgcn_readlane(d, i);
  normalize(dd, fsign, Pc);
  if (j < 12) {
    uint64_t acc = 0;
#pragma unroll
    for (int i = 0; i < NL; i++) {
      const int bit = 30 * i - 32 * (int)j;
      if (bit > -30 && bit < 32) acc |= bit >= 0 ? ((uint64_t)(uint32_t)dd.v[i] << bit) : ((uint64_t)(uint32_t)dd.v[i] >> -bit);
    }
    out[j] = (uint32_t)acc;
  }
}

// ---- the easy part of the final exponentiation, f -> f^((p^6 - 1)(p^2 + 1)), with one Fp
// inversion.  Fp2 products are two dual rows (c0 = a0 b0 + (-a1) b1, c1 = a0 b1 + a1 b0), so
// every step below is ONE round; ws slots [0, 30) hold the intermediate Fp2 values.
__device__ __forceinline__ uint32_t neg128(uint32_t x) { return dfp::sub(0, x, dfp::K_BIAS_NEG); }
// row-th (r < 2 n) component of the Fp2 product of slots (a[i], a[i] + 1) and (b[i], b[i] + 1)
__device__ __forceinline__ uint32_t f2row(const Eng &e, const uint32_t *pa, const uint32_t *pb) {
  const uint32_t j = e.j, k = e.row & 1u;
  const uint32_t a0 = pa[j], a1 = pa[16 + j], b0 = pb[j], b1 = pb[16 + j];
  return k == 0 ? dfp::mul2(a0, b0, neg128(a1), b1, e.t) : dfp::mul2(a0, b1, a1, b0, e.t);
}
// c = f^((p^6 - 1)(p^2 + 1)) (cyclotomic), f != 0; f is kept.  c, t, u: distinct images;
// words: 24 words of LDS.  N = f conj(f) in Fp6; N^-1 = (A, B, C) / F (the adjugate over the
// norm F in Fp2), F^-1 = conj(F) / D with D = F0^2 + F1^2 in Fp inverted by one wave
// (bls_inv.h, variable time: public inputs); then c0 = conj(f)^2 N^-1, c = frob2(c0) c0.
__device__ __forceinline__ void easy_part(Eng &e, uint32_t *c, const uint32_t *f, uint32_t *t,
                                          uint32_t *u, uint32_t *words) {
  uint32_t *ws = e.ws;
  const uint32_t j = e.j, r = e.row;
  conj(e, u, f);
  mul(e, t, f, u);  // N in coefficients 0..5 of t (the w-half is 0 mod p)
  // P0 = n0^2, P1 = n1 n2, P2 = n2^2, P3 = n0 n1, P4 = n1^2, P5 = n0 n2 -> slots 0..11
  if (r < 12) {
    const uint32_t q = r >> 1;
    const uint32_t ia = q == 0 || q == 3 || q == 5 ? 0u : (q == 2 ? 4u : 2u);
    const uint32_t ib = q == 0 ? 0u : (q == 1 || q == 2 || q == 5 ? 4u : 2u);
    ws[16 * r + j] = f2row(e, t + 16 * ia, t + 16 * ib);
  }
  __syncthreads();
  // A = P0 - xi P1, B = xi P2 - P3, C = P4 - P5 (xi (x0 + x1 u) = (x0 - x1) + (x0 + x1) u)
  if (r < 6) {
    const uint32_t *P = ws;
    uint32_t s = dfp::konst(dfp::K_BIAS_R1);
    auto at = [&](int i) { return P[16 * i + j]; };
    switch (r) {
      case 0: s += at(0) + at(3) - at(2); break;
      case 1: s += at(1) - at(2) - at(3); break;
      case 2: s += at(4) - at(5) - at(6); break;
      case 3: s += at(4) + at(5) - at(7); break;
      case 4: s += at(8) - at(10); break;
      default: s += at(9) - at(11); break;
    }
    ws[16 * (12 + r) + j] = dfp::norm(s);
  }
  __syncthreads();
  // T1 = n0 A -> 18, Q1 = n2 B -> 20, Q2 = n1 C -> 22
  if (r < 6) {
    const uint32_t q = r >> 1;
    ws[16 * (18 + r) + j] = f2row(e, t + 16 * (q == 0 ? 0u : (q == 1 ? 4u : 2u)), ws + 16 * (12 + 2 * q));
  }
  __syncthreads();
  // F = T1 + xi (Q1 + Q2) -> 24, 25
  if (r < 2) {
    auto at = [&](int i) { return ws[16 * i + j]; };
    const uint32_t s = r == 0 ? dfp::konst(dfp::K_BIAS_R1) + at(18) + at(20) + at(22) - at(21) - at(23)
                              : at(19) + at(20) + at(22) + at(21) + at(23);
    ws[16 * (24 + r) + j] = dfp::norm(s);
  }
  __syncthreads();
  // D = F0^2 + F1^2 -> canonical words
  if (r == 0) {
    const uint32_t f0 = ws[16 * 24 + j], f1 = ws[16 * 25 + j];
    dfp::to_words(words, dfp::mul2(f0, f0, f1, f1, e.t), e.t);
  }
  __syncthreads();
#if !defined(GBLS_FEXP_NOINV)  // (timing experiment: wrong verdicts without it)
  if (threadIdx.x < 64) inv_wave(words + 12, words);  // wave 0
#endif
  __syncthreads();
  // F^-1 = (F0 d, -F1 d) -> 26, 27 (d = D^-1: the lane's limbs of D^-1 2^-384, times 2^1280)
  if (r < 2) {
    const uint32_t d = dfp::mul(dfp::from_words_scaled(words + 12), dfp::konst(dfp::K_INVFIX), e.t);
    const uint32_t x = ws[16 * (24 + r) + j];
    ws[16 * (26 + r) + j] = dfp::mul(r == 0 ? x : neg128(x), d, e.t);
  }
  __syncthreads();
  // N^-1 = (A, B, C) F^-1 -> t (coefficients 0..5; the w-half zero)
  if (r < 12) t[16 * r + j] = r < 6 ? f2row(e, ws + 16 * (12 + 2 * (r >> 1)), ws + 16 * 26) : 0u;
  __syncthreads();
  mul(e, c, u, u);
  mul(e, c, c, t);
  frob2(e, t, c);
  mul(e, c, c, t);
}
// flags[r] (r < 12) = coefficient r of a minus (r == 0) is 0 mod p: a == 1 iff every flag
__device__ __forceinline__ void one_flags(Eng &e, int *flags, const uint32_t *a) {
  if (e.row < 12) {
    uint32_t x = a[16 * e.row + e.j];
    if (e.row == 0) x = dfp::sub(x, dfp::konst(dfp::K_ONE), dfp::K_BIAS_NEG);
    const bool z = dfp::is_zero(x, e.t);
    if (e.j == 0) flags[e.row] = z ? 1 : 0;
  }
  __syncthreads();
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
