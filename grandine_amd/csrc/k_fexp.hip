// gfx950 kernel: per segment, the product of the Miller partials of every shard (one
// per GPU after the RCCL all-gather, layout [part][segment]), the final
// exponentiation on the wave-cooperative Fp12 engine, and the verdict
// (blst PAIRING_FinalVerify: result == 1, and no set flagged bad), inversion-free.
#include "bls_wave12.h"
#include "bls_w12d.h"
#include "gbls_common.h"

namespace gbls {

// Inversion-free verdict.  f^((p^12-1)/r) == 1 is tested without the easy part's
// f^-1: with G = f^(p^2+1) (= frob2(f) f) and Psi the hard-part chain below -- products,
// Frobenius maps and conj, where conj(y) = y^(p^6) for EVERY y, so Psi(y) = y^e for one
// fixed integer e and Psi commutes with conj -- the cyclotomic element
// F = G^(p^6-1) satisfies Psi(F) = F^(3 (p^4-p^2+1)/r) (the chain's exponent on the
// cyclotomic subgroup) and Psi(F) = Psi(G)^(p^6-1) = conj(Psi(G)) / Psi(G).  Hence
//   f^(3 (p^12-1)/r) == 1   <=>   conj(Psi(G)) == Psi(G)   <=>   Psi(G) has zero w-half,
// for f != 0 (f = 0, a degenerate Miller value, is rejected).  The chain's squarings
// are generic Fp12 squarings (G is not in the cyclotomic subgroup).
__global__ void __launch_bounds__(64) k_final_verdict(const fp12 *part, const int32_t *err,
                                                      uint32_t nparts, uint32_t nseg,
                                                      int32_t *verdict, const uint32_t *lim,
                                                      uint32_t base, const uint32_t *scatter) {
  W12_SHARED uint32_t f[W12_WORDS], G[W12_WORDS], A[W12_WORDS], B[W12_WORDS], T[W12_WORDS],
      X[W12_WORDS], ws[W12_WS_WORDS];
  __shared__ int bad;
  int lane = threadIdx.x;
  uint32_t s = blockIdx.x;
  if (lim && base + s >= *lim) return;  // block-uniform
  w12_plan pl;
  w12_begin(pl, ws);
  const uint32_t *src = reinterpret_cast<const uint32_t *>(part + s);
  for (int i = lane; i < W12_WORDS; i += 64) f[i] = src[i];
  if (lane == 0) bad = err[s];
  __syncthreads();
  for (uint32_t k2 = 1; k2 < nparts; k2++) {
    src = reinterpret_cast<const uint32_t *>(part + (size_t)k2 * nseg + s);
    for (int i = lane; i < W12_WORDS; i += 64) X[i] = src[i];
    if (lane == 0) bad |= err[(size_t)k2 * nseg + s];
    __syncthreads();
    w12_mul(pl, f, f, X, ws);
  }
  if (lane == 0 && w12_is_zero_image(f)) bad = 1;
  // G = f^(p^2+1)
  w12_frob2(G, f);
  w12_mul(pl, G, G, f, ws);
  // A = G^(x-1) = G^x conj(G);  A = A^(x-1)
  w12_exp_x(pl, A, G, ws);
  w12_conj(X, G);
  w12_mul(pl, A, A, X, ws);
  w12_exp_x(pl, B, A, ws);
  w12_conj(X, A);
  w12_mul(pl, A, B, X, ws);
  // B = A^(x+p) = A^x frob(A)
  w12_exp_x(pl, B, A, ws);
  w12_frob(X, A);
  w12_mul(pl, B, B, X, ws);
  // T = B^x;  C = T^x frob2(B) conj(B)   (C in A)
  w12_exp_x(pl, T, B, ws);
  w12_exp_x(pl, A, T, ws);
  w12_frob2(X, B);
  w12_mul(pl, A, A, X, ws);
  w12_conj(X, B);
  w12_mul(pl, A, A, X, ws);
  // R = C G^3
  w12_mul(pl, X, G, G, ws);
  w12_mul(pl, X, X, G, ws);
  w12_mul(pl, A, A, X, ws);
  if (lane == 0)
    verdict[scatter ? scatter[base + s] : s] = (!bad && w12_is_fp6_image(A)) ? ST_SUCCESS : ST_VERIFY_FAIL;
}

// The verdict on the row-distributed Fp12 engine (bls_w12d.h): one 56-row workgroup per
// segment, every Fp12 product one row-product deep.  The latency form, for launches of a few
// segments (blocks, gossip batches, C2 batches), where the one-wave form leaves the chip idle
// behind a serial chain of ~350 Fp12 operations.  Partials are read as repacked limbs (an Fp*
// scalar per partial, which the exponentiation removes).
//
// Unlike the one-wave form this one pays for the easy part's inversion (one Fp inversion on
// one lane, bls_inv.h, plus a few Fp2 rounds): m = f^((p^6 - 1)(p^2 + 1)) is then in the
// cyclotomic subgroup, the hard part's ~315 squarings are Granger-Scott squarings (18 row
// products and one combine round, against 36 and two), and the verdict is the textbook one:
// m^(3 (p^4 - p^2 + 1) / r) == 1 (the chain's exponent; gcd(3, r) = 1, so this is
// f^((p^12 - 1) / r) == 1, blst's PAIRING_FinalVerify).
__global__ void __launch_bounds__(w12d::THREADS) k_final_verdict_d(const fp12 *part,
                                                                   const int32_t *err,
                                                                   uint32_t nparts, uint32_t nseg,
                                                                   int32_t *verdict, const uint32_t *lim,
                                                                   uint32_t base, const uint32_t *scatter) {
  __shared__ __attribute__((aligned(16))) uint32_t f[w12d::IMG], G[w12d::IMG], A[w12d::IMG],
      B[w12d::IMG], T[w12d::IMG], X[w12d::IMG], ws[w12d::WS], words[24];
  __shared__ int flags[12];
  __shared__ int bad;
  const uint32_t s = blockIdx.x;
  if (lim && base + s >= *lim) return;  // block-uniform
  w12d::Eng e;
  w12d::begin(e, ws);
  w12d::load_scaled(e, f, reinterpret_cast<const uint32_t *>(part + s));
  if (threadIdx.x == 0) bad = err[s];
  for (uint32_t k2 = 1; k2 < nparts; k2++) {
    w12d::load_scaled(e, X, reinterpret_cast<const uint32_t *>(part + (size_t)k2 * nseg + s));
    if (threadIdx.x == 0) bad |= err[(size_t)k2 * nseg + s];
    w12d::mul(e, f, f, X);
  }
  w12d::zero_flags(e, flags, f, 0, 12);  // f = 0 (a degenerate Miller value) is rejected
  if (threadIdx.x == 0) {
    int all = 1;
    for (int i = 0; i < 12; i++) all &= flags[i];
    if (all) bad = 1;
  }
  // G = f^((p^6 - 1)(p^2 + 1)); A = G^(x-1); A = A^(x-1); B = A^(x+p);
  // C = B^(x^2) frob2(B) conj(B); R = C G^3 (the k_final_verdict chain, same exponents; conj
  // is the inverse on the cyclotomic subgroup)
  w12d::easy_part(e, G, f, T, X, words);
#if defined(GBLS_FEXP_EASY_ONLY)  // timing experiment
  if (threadIdx.x == 0) verdict[s] = G[0] == 12345u ? 1 : 0;
  return;
#endif
  w12d::exp_x_cyc(e, A, G);
  w12d::conj(e, X, G);
  w12d::mul(e, A, A, X);
  w12d::exp_x_cyc(e, B, A);
  w12d::conj(e, X, A);
  w12d::mul(e, A, B, X);
  w12d::exp_x_cyc(e, B, A);
  w12d::frob(e, X, A);
  w12d::mul(e, B, B, X);
  w12d::exp_x_cyc(e, T, B);
  w12d::exp_x_cyc(e, A, T);
  w12d::frob2(e, X, B);
  w12d::mul(e, A, A, X);
  w12d::conj(e, X, B);
  w12d::mul(e, A, A, X);
  w12d::cyc_sqr(e, X, G);
  w12d::mul(e, X, X, G);
  w12d::mul(e, A, A, X);
  w12d::one_flags(e, flags, A);  // R == 1
  if (threadIdx.x == 0) {
    int one = 1;
    for (int i = 0; i < 12; i++) one &= flags[i];
    verdict[scatter ? scatter[base + s] : s] = (!bad && one) ? ST_SUCCESS : ST_VERIFY_FAIL;
  }
}

// segments up to this many take the row-distributed (latency) form
constexpr uint32_t kFinalRowsMaxSegs = 64;

void launch_final_verdict(hipStream_t st, const fp12 *partials, const int32_t *err,
                          uint32_t nparts, uint32_t nseg, int32_t *verdict, const uint32_t *lim,
                          uint32_t base, const uint32_t *scatter) {
  if (!nseg) return;
  if (nseg <= kFinalRowsMaxSegs)
    k_final_verdict_d<<<nseg, w12d::THREADS, 0, st>>>(partials, err, nparts, nseg, verdict, lim, base,
                                                       scatter);
  else
    k_final_verdict<<<nseg, 64, 0, st>>>(partials, err, nparts, nseg, verdict, lim, base, scatter);
}

}  // namespace gbls
