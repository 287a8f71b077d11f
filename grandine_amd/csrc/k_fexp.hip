// gfx950 kernel: per segment, the product of the Miller partials of every shard (one
// per GPU after the RCCL all-gather, layout [part][segment]), the final
// exponentiation on the wave-cooperative Fp12 engine, and the verdict
// (blst PAIRING_FinalVerify: result == 1, and no set flagged bad), inversion-free.
#include "bls_wave12.h"
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
                                                      int32_t *verdict) {
  W12_SHARED uint32_t f[W12_WORDS], G[W12_WORDS], A[W12_WORDS], B[W12_WORDS], T[W12_WORDS],
      X[W12_WORDS], ws[W12_WS_WORDS];
  __shared__ int bad;
  int lane = threadIdx.x;
  w12_plan pl;
  w12_begin(pl, ws);
  uint32_t s = blockIdx.x;
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
  if (lane == 0) verdict[s] = (!bad && w12_is_fp6_image(A)) ? ST_SUCCESS : ST_VERIFY_FAIL;
}

void launch_final_verdict(hipStream_t st, const fp12 *partials, const int32_t *err,
                          uint32_t nparts, uint32_t nseg, int32_t *verdict) {
  if (nseg) k_final_verdict<<<nseg, 64, 0, st>>>(partials, err, nparts, nseg, verdict);
}

}  // namespace gbls
