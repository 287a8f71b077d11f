// Row-distributed Fp arithmetic for the latency regime (VERDICT r02 "next 1b": the limb-split
// product).  One element of the BLS12-381 base field is spread over a 16-lane DPP row: lane j
// holds limb j of x = sum_j l_j 2^(28 j), in Montgomery form with R = 2^448 (16 limbs of 28
// bits; p needs 14).  An element is ONE register per lane, additions are lane-local (no carry
// chain), and a Montgomery product costs ~220 instructions per lane instead of the ~690 of the
// engine's one-lane product (bls_fpmul_gen.h): the latency of a serial chain (the final
// exponentiation, the Horner step over the Miller events, square-root exponentiations) drops
// by ~3x, paid for with 16 lanes per product.  Cross-lane traffic is DPP only (row_newbcast,
// row_shr / row_shl / row_ror): VALU moves, no LDS, no barrier.
//
// Limb and value contract ("almost normalized": the output of norm / mul):
//   limbs in [0, 2^28 + 2^9), limbs 14 and 15 zero whenever the value is < 2^392;
//   mul inputs: limbs < 2^29 and value < 2^392 (~2^10.6 p); output value < p + 2^336;
//   lazy sums of k almost-normalized elements need one norm() pass (limbs < 2^28 + 2k) before
//   they feed a product.
// Subtraction adds a multiple of p whose lower limbs are pre-borrowed (bls_dfp_tables.h
// K_BIAS*), so no limb ever goes negative.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "bls_constants.h"
#include "bls_dfp_tables.h"

namespace gbls {
namespace dfp {

constexpr uint32_t M28 = 0x0fffffffu;

// ---- DPP row primitives (16-lane rows; gfx9 dpp_ctrl encodings)
template <int N>
__device__ __forceinline__ uint32_t bcast(uint32_t v) {  // every lane <- lane N of its row
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x150 + N, 0xf, 0xf, false);
}
template <int N>
__device__ __forceinline__ uint32_t shr(uint32_t v) {  // lane j <- lane j - N, 0 for j < N
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x110 + N, 0xf, 0xf, true);
}
template <int N>
__device__ __forceinline__ uint32_t shl(uint32_t v) {  // lane j <- lane j + N, 0 for j + N > 15
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x100 + N, 0xf, 0xf, true);
}
template <int N>
__device__ __forceinline__ uint32_t ror(uint32_t v) {  // lane j <- lane (j - N) mod 16
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x120 + N, 0xf, 0xf, false);
}

// compile-time loop
template <int I, int E>
struct For {
  template <class F>
  __device__ __forceinline__ static void run(F &&f) {
    f(std::integral_constant<int, I>());
    For<I + 1, E>::run(f);
  }
};
template <int E>
struct For<E, E> {
  template <class F>
  __device__ __forceinline__ static void run(F &&) {}
};

// The lane's limb index; the product's constants (p, p') are wave-uniform and live in SGPRs.
struct Tabs {
  uint32_t j;
};
__device__ __forceinline__ void load_tabs(Tabs &t) { t.j = threadIdx.x & 15; }
// the lane's limb of a constant (K_* tables)
__device__ __forceinline__ uint32_t konst(const uint32_t (&k)[16]) { return k[threadIdx.x & 15]; }

// ---- carry handling
// One pass on a 64-bit column: low 28 bits stay, the rest moves one lane up (mod 2^448: the
// carry out of lane 15 is dropped).  Limbs < 2^64 -> < 2^28 + 2^36.
__device__ __forceinline__ uint64_t pass64(uint64_t x) {
  const uint64_t c = x >> 28;
  const uint32_t c0 = shr<1>((uint32_t)c), c1 = shr<1>((uint32_t)(c >> 32));
  return (x & M28) + (((uint64_t)c1 << 32) | c0);
}
// One pass on 32-bit limbs: limbs < 2^32 -> < 2^28 + 2^4 (top carry dropped)
__device__ __forceinline__ uint32_t norm(uint32_t x) { return (x & M28) + shr<1>(x >> 28); }
// 64-bit columns -> almost-normalized 32-bit limbs, mod 2^448
__device__ __forceinline__ uint32_t norm64(uint64_t x) {
  x = pass64(x);                     // < 2^28 + 2^36
  const uint32_t lo = (uint32_t)x;   // x < 2^37: the shift below sees every bit
  const uint32_t c = (uint32_t)(x >> 28);
  return (lo & M28) + shr<1>(c);     // < 2^28 + 2^9
}
// Passes over the low half of a product, whose carry out of lane 15 belongs to column 16,
// i.e. to lane 0's high column: the carries rotate (row_ror) and lane 0 adds its incoming
// carry to `hi` instead of `lo`.
__device__ __forceinline__ void pass_lo64(uint64_t &lo, uint64_t &hi, uint32_t j) {
  const uint64_t c = lo >> 28;
  const uint32_t c0 = ror<1>((uint32_t)c), c1 = ror<1>((uint32_t)(c >> 32));
  const uint64_t cin = ((uint64_t)c1 << 32) | c0;
  lo &= M28;
  const uint64_t zero = 0;
  lo += j ? cin : zero;
  hi += j ? zero : cin;
}
__device__ __forceinline__ void pass_lo32(uint64_t &lo, uint64_t &hi, uint32_t j) {
  const uint32_t c = ror<1>((uint32_t)(lo >> 28));  // lo < 2^37
  lo &= M28;
  lo += j ? c : 0u;
  hi += j ? 0u : c;
}

// T += a b: lane j accumulates column j (lo) and column j + 16 (hi).  a, b have 14 limbs.
// Odd and even terms go to separate accumulators (GBLS_DFP_ONE_ACC: one chain), so the 64-bit
// multiply-adds form two independent dependency chains: a lone wave (the latency regime's
// chains) otherwise waits on every accumulate.
__device__ __forceinline__ void columns(uint64_t &lo, uint64_t &hi, uint32_t a, uint32_t b) {
#if defined(GBLS_DFP_ONE_ACC)
  lo += (uint64_t)bcast<0>(a) * b;
  For<1, 14>::run([&](auto I) {
    constexpr int i = decltype(I)::value;
    const uint32_t ai = bcast<i>(a);
    lo += (uint64_t)ai * shr<i>(b);       // b_(j-i), j >= i
    hi += (uint64_t)ai * shl<16 - i>(b);  // b_(j+16-i), j < i
  });
#else
  uint64_t lo1 = 0, hi1 = 0;
  lo += (uint64_t)bcast<0>(a) * b;
  For<1, 14>::run([&](auto I) {
    constexpr int i = decltype(I)::value;
    const uint32_t ai = bcast<i>(a);
    if constexpr (i & 1) {
      lo1 += (uint64_t)ai * shr<i>(b);       // b_(j-i), j >= i
      hi1 += (uint64_t)ai * shl<16 - i>(b);  // b_(j+16-i), j < i
    } else {
      lo += (uint64_t)ai * shr<i>(b);
      hi += (uint64_t)ai * shl<16 - i>(b);
    }
  });
  lo += lo1;
  hi += hi1;
#endif
}
__device__ __forceinline__ uint32_t redc(uint64_t lo, uint64_t hi, const Tabs &t);

// ---- Montgomery product a b / 2^448 mod p (see the contract above)
__device__ __forceinline__ uint32_t mul(uint32_t a, uint32_t b, const Tabs &t) {
  uint64_t lo = 0, hi = 0;
  columns(lo, hi, a, b);
  return redc(lo, hi, t);
}
// (a b + c d) / 2^448 mod p in one reduction (column sums < 2 x 14 x 2^58 < 2^63); output
// < p + 2^337
__device__ __forceinline__ uint32_t mul2(uint32_t a, uint32_t b, uint32_t c, uint32_t d,
                                         const Tabs &t) {
  uint64_t lo = 0, hi = 0;
  columns(lo, hi, a, b);
  columns(lo, hi, c, d);
  return redc(lo, hi, t);
}
// Montgomery reduction of the column sums of T (lo: columns 0..15, hi: 16..31)
__device__ __forceinline__ uint32_t redc(uint64_t lo, uint64_t hi, const Tabs &t) {
  const uint32_t j = t.j;
  // T_lo to limbs < 2^29 (its carries flow into column 16 = lane 0's hi)
  pass_lo64(lo, hi, j);
  pass_lo32(lo, hi, j);
  const uint32_t tl = (uint32_t)lo;
  // m = T_lo p' mod 2^448: column j = sum over i <= j of p'_i t_(j-i)
#if defined(GBLS_DFP_ONE_ACC)
  uint64_t mc = (uint64_t)K_PINV_U[0] * tl;
  For<1, 16>::run([&](auto I) {
    constexpr int i = decltype(I)::value;
    mc += (uint64_t)K_PINV_U[i] * shr<i>(tl);
  });
  const uint32_t m = norm64(mc);
  // U = T + m p (p_i uniform, m shifted across the row); U_lo = 0 mod 2^448
  lo += (uint64_t)K_P_U[0] * m;
  For<1, 14>::run([&](auto I) {
    constexpr int i = decltype(I)::value;
    lo += (uint64_t)K_P_U[i] * shr<i>(m);       // m_(j-i), j >= i
    hi += (uint64_t)K_P_U[i] * shl<16 - i>(m);  // m_(j+16-i), j < i
  });
#else
  uint64_t mc = (uint64_t)K_PINV_U[0] * tl, mc1 = 0;
  For<1, 16>::run([&](auto I) {
    constexpr int i = decltype(I)::value;
    if constexpr (i & 1)
      mc1 += (uint64_t)K_PINV_U[i] * shr<i>(tl);
    else
      mc += (uint64_t)K_PINV_U[i] * shr<i>(tl);
  });
  const uint32_t m = norm64(mc + mc1);
  // U = T + m p (p_i uniform, m shifted across the row); U_lo = 0 mod 2^448
  uint64_t lo1 = 0, hi1 = 0;
  lo += (uint64_t)K_P_U[0] * m;
  For<1, 14>::run([&](auto I) {
    constexpr int i = decltype(I)::value;
    if constexpr (i & 1) {
      lo1 += (uint64_t)K_P_U[i] * shr<i>(m);       // m_(j-i), j >= i
      hi1 += (uint64_t)K_P_U[i] * shl<16 - i>(m);  // m_(j+16-i), j < i
    } else {
      lo += (uint64_t)K_P_U[i] * shr<i>(m);
      hi += (uint64_t)K_P_U[i] * shl<16 - i>(m);
    }
  });
  lo += lo1;
  hi += hi1;
#endif
  // carry of U_lo into column 16: after two passes the low limbs are < 2^28 + 2^9 and their
  // value, a multiple of 2^448 below 2^449, is 2^448 exactly when any limb is nonzero
  pass_lo64(lo, hi, j);
  pass_lo32(lo, hi, j);
  const uint64_t nz = __ballot((uint32_t)lo != 0);
  const uint32_t row_nz = (uint32_t)(nz >> (threadIdx.x & 48)) & 0xffffu;
  hi += (j == 0 && row_nz) ? 1u : 0u;
  return norm64(hi);  // the result (< p + 2^336) never carries out of lane 15
}

// ---- lane-local linear operations (see the contract for when norm() is due)
__device__ __forceinline__ uint32_t add(uint32_t a, uint32_t b) { return norm(a + b); }
// bias - b (+ a): bias = K p with its lower limbs pre-borrowed (bls_dfp_tables.h)
__device__ __forceinline__ uint32_t sub(uint32_t a, uint32_t b, const uint32_t (&bias)[16]) {
  return norm(a + konst(bias) - b);
}

// Zero test of a value < 2^392: r = x / 2^448 mod p lies in [0, p + 2^336), so x = 0 mod p
// iff r is 0 or p; the row's limbs of r are gathered into every lane and normalized serially.
// Every lane of the row returns the same answer.
__device__ __forceinline__ bool is_zero(uint32_t x, const Tabs &t) {
  const uint32_t one = (t.j == 0) ? 1u : 0u;
  const uint32_t r = mul(x, one, t);
  uint32_t l[16];
  For<0, 16>::run([&](auto I) {
    constexpr int i = decltype(I)::value;
    l[i] = bcast<i>(r);
  });
  uint32_t c = 0, z = 0, e = 0;
#pragma unroll
  for (int i = 0; i < 16; i++) {
    const uint32_t v = l[i] + c;
    c = v >> 28;
    const uint32_t d = v & M28;
    z |= d;
    e |= d ^ K_P[i];
  }
  return z == 0 || e == 0;
}

// Engine form (12 x 32-bit words, x 2^384 mod p) -> this form (x 2^448): lane j takes bits
// [28 j, 28 j + 28) of the 384-bit word string and the row multiplies by 2^512 mod p.
__device__ __forceinline__ uint32_t from_words(const uint32_t *w, const Tabs &t) {
  const uint32_t j = t.j;
  uint32_t v = 0;
  if (j < 14) {
    const uint32_t bit = 28 * j, k = bit >> 5, s = bit & 31;
    uint64_t pair = w[k];
    if (k + 1 < 12) pair |= (uint64_t)w[k + 1] << 32;
    v = (uint32_t)(pair >> s) & M28;
  }
  return mul(v, konst(K_CIN), t);
}
// The repacked 28-bit limbs of engine-form words WITHOUT the conversion product: the same
// element times 2^-64 in this form (a nonzero Fp scalar, which the final exponentiation
// removes -- only for Miller values).
__device__ __forceinline__ uint32_t from_words_scaled(const uint32_t *w) {
  const uint32_t j = threadIdx.x & 15;
  uint32_t v = 0;
  if (j < 14) {
    const uint32_t bit = 28 * j, k = bit >> 5, s = bit & 31;
    uint64_t pair = w[k];
    if (k + 1 < 12) pair |= (uint64_t)w[k + 1] << 32;
    v = (uint32_t)(pair >> s) & M28;
  }
  return v;
}
// This form -> canonical engine-form words (x 2^384 mod p, < p): the row multiplies by
// 2^384 mod p, every lane gathers and normalizes the limbs, subtracts p once if needed, and
// lane j < 12 returns word j (the other lanes return 0).
__device__ __forceinline__ uint32_t word_of(uint32_t x, const Tabs &t) {
  const uint32_t r = mul(x, konst(K_COUT), t);
  uint32_t l[16];
  For<0, 16>::run([&](auto I) {
    constexpr int i = decltype(I)::value;
    l[i] = bcast<i>(r);
  });
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 16; i++) {
    const uint32_t v = l[i] + c;
    c = v >> 28;
    l[i] = v & M28;
  }
  // subtract p when l >= p (l < p + 2^336 < 2p)
  uint32_t d[16];
  int32_t br = 0;
#pragma unroll
  for (int i = 0; i < 16; i++) {
    const int32_t v = (int32_t)l[i] - (int32_t)K_P[i] + br;
    br = v >> 28;
    d[i] = (uint32_t)v & M28;
  }
  const bool ge = br == 0;
#pragma unroll
  for (int i = 0; i < 16; i++) l[i] = ge ? d[i] : l[i];
  // 28-bit limbs -> 32-bit words; lane j < 12 takes word j
  const uint32_t j = t.j;
  uint32_t word = 0;
  if (j < 12) {
#pragma unroll
    for (int i = 0; i < 14; i++) {
      const int lo_bit = 28 * i - 32 * (int)j;  // position of limb i inside word j
      if (lo_bit > -28 && lo_bit < 32)
        word |= lo_bit >= 0 ? (l[i] << lo_bit) : (l[i] >> -lo_bit);
    }
  }
  return word;
}
// word j of the canonical residue of the row value v = x 2^448 mod p itself, WITHOUT the
// 2^-64 conversion product: read as engine form it is the element x 2^64 (an Fp* scale
// factor -- for Miller line coefficients, which the final exponentiation cleans).  v < 2^392
// (any lazy sum): one estimated multiple of p off (q = top limb / (p_13 + 1)), then at most
// two conditional subtractions.
__device__ __forceinline__ uint32_t word_of_scaled(uint32_t x) {
  uint32_t l[16];
  For<0, 16>::run([&](auto I) {
    constexpr int i = decltype(I)::value;
    l[i] = bcast<i>(x);
  });
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 16; i++) {
    const uint32_t v = l[i] + c;
    c = v >> 28;
    l[i] = v & M28;
  }
  // v < 2^392: limbs 14, 15 are zero; v - q p >= 0 and < p + 2^364 (q <= v / ((p_13 + 1) 2^364))
  const uint32_t q = l[13] / (K_P_U[13] + 1u);
  int64_t br = 0;
#pragma unroll
  for (int i = 0; i < 14; i++) {
    const int64_t v = (int64_t)l[i] - (int64_t)q * K_P_U[i] + br;
    l[i] = (uint32_t)v & M28;
    br = v >> 28;  // arithmetic shift: the borrow
  }
#pragma unroll
  for (int rep = 0; rep < 2; rep++) {
    uint32_t d[14];
    int32_t b2 = 0;
#pragma unroll
    for (int i = 0; i < 14; i++) {
      const int32_t v = (int32_t)l[i] - (int32_t)K_P_U[i] + b2;
      b2 = v >> 28;
      d[i] = (uint32_t)v & M28;
    }
    const bool ge = b2 == 0;
#pragma unroll
    for (int i = 0; i < 14; i++) l[i] = ge ? d[i] : l[i];
  }
  const uint32_t j = threadIdx.x & 15;
  uint32_t word = 0;
  if (j < 12) {
#pragma unroll
    for (int i = 0; i < 14; i++) {
      const int lo_bit = 28 * i - 32 * (int)j;
      if (lo_bit > -28 && lo_bit < 32) word |= lo_bit >= 0 ? (l[i] << lo_bit) : (l[i] >> -lo_bit);
    }
  }
  return word;
}
__device__ __forceinline__ void to_words(uint32_t *w, uint32_t x, const Tabs &t) {
  const uint32_t word = word_of(x, t);
  if (t.j < 12) w[t.j] = word;
}

// The row form (x 2^448) of an engine-form value held IN REGISTERS by every lane of the row
// (x 2^384, 12 words): lane j selects its limb with constant indices (no dynamic register
// indexing), then the row multiplies by 2^512 mod p.
__device__ __forceinline__ uint32_t from_regs(const uint32_t (&w)[12], const Tabs &t) {
  uint32_t v = 0;
#pragma unroll
  for (int i = 0; i < 14; i++) {
    const int bit = 28 * i, k = bit >> 5, sh = bit & 31;
    uint64_t pair = w[k];
    if (k + 1 < 12) pair |= (uint64_t)w[k + 1] << 32;
    const uint32_t limb = (uint32_t)(pair >> sh) & M28;
    v = t.j == (uint32_t)i ? limb : v;
  }
  return mul(v, konst(K_CIN), t);
}

// x^((p-3)/4) on the row: the engine's sliding-window schedule (bls_constants.h PM3D4_*,
// ~379 squarings + 79 products), the 8 odd powers in registers (one per lane each).
__device__ __forceinline__ uint32_t pow_pm3d4(uint32_t x, const Tabs &t) {
  uint32_t tab[8];
  const uint32_t x2 = mul(x, x, t);
  tab[0] = x;
#pragma unroll
  for (int i = 1; i < 8; i++) tab[i] = mul(tab[i - 1], x2, t);
  uint32_t acc = tab[k::PM3D4_TOP >> 1];
  for (int e = 0; e < k::PM3D4_NWIN; e++) {
    const int sq = k::PM3D4_WIN[e][0], d = k::PM3D4_WIN[e][1];
    for (int i = 0; i < sq; i++) acc = mul(acc, acc, t);
    if (d) {
      uint32_t y = tab[0];
#pragma unroll
      for (int i = 1; i < 8; i++) y = (d >> 1) == i ? tab[i] : y;  // no dynamic register index
      acc = mul(acc, y, t);
    }
  }
  return acc;
}

// Every lane of the row gets the canonical engine-form words (x 2^384 mod p, < p) of x.
__device__ __forceinline__ void to_words_all(uint32_t (&w)[12], uint32_t x, const Tabs &t) {
  const uint32_t r = mul(x, konst(K_COUT), t);
  uint32_t l[16];
  For<0, 16>::run([&](auto I) {
    constexpr int i = decltype(I)::value;
    l[i] = bcast<i>(r);
  });
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 16; i++) {
    const uint32_t v = l[i] + c;
    c = v >> 28;
    l[i] = v & M28;
  }
  uint32_t d[16];
  int32_t br = 0;
#pragma unroll
  for (int i = 0; i < 16; i++) {
    const int32_t v = (int32_t)l[i] - (int32_t)K_P[i] + br;
    br = v >> 28;
    d[i] = (uint32_t)v & M28;
  }
  const bool ge = br == 0;
#pragma unroll
  for (int i = 0; i < 16; i++) l[i] = ge ? d[i] : l[i];
  uint64_t buf = 0;
  int have = 0, k = 0;
#pragma unroll
  for (int i = 0; i < 14; i++) {
    buf |= (uint64_t)l[i] << have;
    have += 28;
    if (have >= 32 && k < 12) {  // 14 limbs = 392 bits; the canonical value fits 12 words
      w[k++] = (uint32_t)buf;
      buf >>= 32;
      have -= 32;
    }
  }
}

}  // namespace dfp
}  // namespace gbls
