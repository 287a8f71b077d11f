// Fast variable-time inversion in Fp (bls_field.h fp_inv: the lane kernels' affine
// conversions, the final exponentiation's easy part in bls_w12d.h): Bernstein-Yang
// "safegcd" divsteps in batches of 30 on signed 30-bit limbs, the variable-time form
// (batches of zero-skipping and cancelling steps).  ~26 batches for a 381-bit input, each a few
// hundred 32-bit instructions (signed 32x32 -> 64-bit mads for the matrix updates).
// Every input on the verification path is public, so variable time is fine.
//
// Same contract as fp_inv: Montgomery form in (a R), Montgomery form out (a^-1 R), 0 -> 0.
//
// Attribution: the structure follows the public variable-time safegcd of libsecp256k1
// (src/modinv32_impl.h, MIT licence: secp256k1_modinv32_var with its divsteps_30_var /
// update_de_30 / update_fg_30_var decomposition and the ctz(g | (~0 << i)) zero-skipping loop),
// itself an implementation of D. J. Bernstein and B.-Y. Yang, "Fast constant-time gcd
// computation and modular inversion" (TCHES 2019).  Re-targeted here to 13 x 30-bit limbs of the
// BLS12-381 base field and to the engine's Montgomery form; not code of the reference repository.
#pragma once
#include "bls_field.h"

namespace gbls {
namespace binv {

constexpr int NL = 13;  // 13 x 30 bits = 390 >= 381 (+ sign headroom in the top limb)
constexpr int32_t M30 = 0x3fffffff;

struct S30 {
  int32_t v[NL];
};
struct Mat {
  int32_t u, v, q, r;
};

// p in signed 30-bit limbs and p^-1 mod 2^30 (computed once from k::P by the callers' constant
// folding: pure integer functions of the 32-bit words)
HD void p30(S30 &m) {
#pragma unroll
  for (int i = 0; i < NL; i++) {
    const int bit = 30 * i, w = bit >> 5, s = bit & 31;
    uint64_t pair = k::P[w];
    if (w + 1 < 12) pair |= (uint64_t)k::P[w + 1] << 32;
    m.v[i] = (int32_t)((pair >> s) & (uint64_t)M30);
  }
}
HD uint32_t inv32(uint32_t a) {  // a^-1 mod 2^32 for odd a (Newton: 3 -> 6 -> 12 -> 24 -> 48 bits)
  uint32_t x = a;                // a a = 1 mod 8
  x *= 2u - a * x;
  x *= 2u - a * x;
  x *= 2u - a * x;
  x *= 2u - a * x;
  return x;
}

// 30 divsteps on the low bits of f (odd) and g; returns the new eta, the transition matrix
// scaled by 2^30 in t.  (eta = -delta; the matrix entries end up in [-2^30, 2^30].)
HD int32_t divsteps30(int32_t eta, uint32_t f, uint32_t g, Mat &t) {
  uint32_t u = 1, v = 0, q = 0, r = 1;
  int i = 30;
  for (;;) {
    // zeros of g, counted up to i (a sentinel bit at position i)
    const int zeros = __builtin_ctz(g | (0xffffffffu << i));
    g >>= zeros;
    u <<= zeros;
    v <<= zeros;
    eta -= zeros;
    i -= zeros;
    if (i == 0) break;
    if (eta < 0) {  // swap: (f, g) <- (g, -f), with the matrix rows
      eta = -eta;
      uint32_t tmp = f;
      f = g;
      g = 0u - tmp;
      tmp = u;
      u = q;
      q = 0u - tmp;
      tmp = v;
      v = r;
      r = 0u - tmp;
    }
    // cancel the low min(eta + 1, i) bits of g with a multiple of f (f odd)
    const int limit = (eta + 1) > i ? i : (eta + 1);
    const uint32_t m = 0xffffffffu >> (32 - limit);
    const uint32_t w = (0u - g * inv32(f)) & m;
    g += f * w;
    q += u * w;
    r += v * w;
  }
  t.u = (int32_t)u;
  t.v = (int32_t)v;
  t.q = (int32_t)q;
  t.r = (int32_t)r;
  return eta;
}

// [d, e] <- t [d, e] / 2^30 mod p (d, e in (-2p, p) stay there)
HD void update_de(S30 &d, S30 &e, const Mat &t, const S30 &P, uint32_t pinv30) {
  const int32_t u = t.u, v = t.v, q = t.q, r = t.r;
  const int32_t sd = d.v[NL - 1] >> 31, se = e.v[NL - 1] >> 31;
  int32_t md = (u & sd) + (v & se), me = (q & sd) + (r & se);
  int64_t cd = (int64_t)u * d.v[0] + (int64_t)v * e.v[0];
  int64_t ce = (int64_t)q * d.v[0] + (int64_t)r * e.v[0];
  md -= (int32_t)((pinv30 * (uint32_t)cd + (uint32_t)md) & (uint32_t)M30);
  me -= (int32_t)((pinv30 * (uint32_t)ce + (uint32_t)me) & (uint32_t)M30);
  cd += (int64_t)P.v[0] * md;
  ce += (int64_t)P.v[0] * me;
  cd >>= 30;
  ce >>= 30;
#pragma unroll
  for (int i = 1; i < NL; i++) {
    const int32_t di = d.v[i], ei = e.v[i];
    cd += (int64_t)u * di + (int64_t)v * ei + (int64_t)P.v[i] * md;
    ce += (int64_t)q * di + (int64_t)r * ei + (int64_t)P.v[i] * me;
    d.v[i - 1] = (int32_t)cd & M30;
    cd >>= 30;
    e.v[i - 1] = (int32_t)ce & M30;
    ce >>= 30;
  }
  d.v[NL - 1] = (int32_t)cd;
  e.v[NL - 1] = (int32_t)ce;
}

// [f, g] <- t [f, g] / 2^30 (exact division).  Always over all NL limbs: with the operand
// length shrinking as the values do, the limb arrays were indexed by a run-time length and
// the compiler kept them in scratch memory (56 B per lane in every kernel with an inversion).
HD void update_fg(S30 &f, S30 &g, const Mat &t) {
  const int32_t u = t.u, v = t.v, q = t.q, r = t.r;
  int64_t cf = (int64_t)u * f.v[0] + (int64_t)v * g.v[0];
  int64_t cg = (int64_t)q * f.v[0] + (int64_t)r * g.v[0];
  cf >>= 30;
  cg >>= 30;
#pragma unroll
  for (int i = 1; i < NL; i++) {
    const int32_t fi = f.v[i], gi = g.v[i];
    cf += (int64_t)u * fi + (int64_t)v * gi;
    cg += (int64_t)q * fi + (int64_t)r * gi;
    f.v[i - 1] = (int32_t)cf & M30;
    cf >>= 30;
    g.v[i - 1] = (int32_t)cg & M30;
    cg >>= 30;
  }
  f.v[NL - 1] = (int32_t)cf;
  g.v[NL - 1] = (int32_t)cg;
}

// r in (-2p, p) -> r (or -r when sign < 0) in [0, p)
HD void normalize(S30 &r, int32_t sign, const S30 &P) {
  int32_t add = r.v[NL - 1] >> 31;
#pragma unroll
  for (int i = 0; i < NL; i++) r.v[i] += P.v[i] & add;
  const int32_t neg = sign >> 31;
#pragma unroll
  for (int i = 0; i < NL; i++) r.v[i] = (r.v[i] ^ neg) - neg;
#pragma unroll
  for (int i = 0; i < NL - 1; i++) {
    r.v[i + 1] += r.v[i] >> 30;
    r.v[i] &= M30;
  }
  add = r.v[NL - 1] >> 31;
#pragma unroll
  for (int i = 0; i < NL; i++) r.v[i] += P.v[i] & add;
#pragma unroll
  for (int i = 0; i < NL - 1; i++) {
    r.v[i + 1] += r.v[i] >> 30;
    r.v[i] &= M30;
  }
}

// x^-1 mod p of the plain integer x (12 little-endian words, 0 < x, gcd(x, p) = 1)
HD void inverse_words(uint32_t (&out)[12], const uint32_t (&x)[12]) {
  S30 P, d, e, f, g;
  p30(P);
  const uint32_t pinv30 = inv32((uint32_t)P.v[0]) & (uint32_t)M30;
#pragma unroll
  for (int i = 0; i < NL; i++) {
    const int bit = 30 * i, w = bit >> 5, s = bit & 31;
    uint64_t pair = x[w];
    if (w + 1 < 12) pair |= (uint64_t)x[w + 1] << 32;
    g.v[i] = (int32_t)((pair >> s) & (uint64_t)M30);
    d.v[i] = 0;
    e.v[i] = i == 0 ? 1 : 0;
    f.v[i] = P.v[i];
  }
  int32_t eta = -1;
  for (int guard = 0; guard < 64; guard++) {  // ~26 batches for 381 bits; bound ~37
    Mat t;
    eta = divsteps30(eta, (uint32_t)f.v[0], (uint32_t)g.v[0], t);
    update_de(d, e, t, P, pinv30);
    update_fg(f, g, t);
    int32_t any = 0;
#pragma unroll
    for (int j = 0; j < NL; j++) any |= g.v[j];
    if (any == 0) break;
  }
  // f = +-1 (gcd 1): d = +-x^-1
  normalize(d, f.v[NL - 1], P);
#pragma unroll
  for (int k2 = 0; k2 < 12; k2++) {
    uint64_t acc = 0;
#pragma unroll
    for (int i = 0; i < NL; i++) {
      const int bit = 30 * i - 32 * k2;
      if (bit > -30 && bit < 32) acc |= bit >= 0 ? ((uint64_t)(uint32_t)d.v[i] << bit) : ((uint64_t)(uint32_t)d.v[i] >> -bit);
    }
    out[k2] = (uint32_t)acc;
  }
}

}  // namespace binv

// a^-1 R from a R (Montgomery, R = 2^384); 0 -> 0
HD void fp_inv_var(fp &r, const fp &a) {
  if (fp_is_zero(a)) {
    fp_zero(r);
    return;
  }
  uint32_t x[12], y[12];
#pragma unroll
  for (int i = 0; i < 12; i++) x[i] = a.l[i];
  binv::inverse_words(y, x);
  fp t;
#pragma unroll
  for (int i = 0; i < 12; i++) t.l[i] = y[i];
  fp_mul(r, t, fp_const(k::R3));  // (aR)^-1 R^3 / R = a^-1 R
}

}  // namespace gbls
