// gfx950 kernel: per segment, the product of the Miller partials of every shard (one
// per GPU after the RCCL all-gather, layout [part][segment]), the final
// exponentiation on the wave-cooperative Fp12 engine, and the verdict
// (blst PAIRING_FinalVerify: result == 1, and no set flagged bad).
#include "bls_wave12.h"
#include "gbls_common.h"

namespace gbls {

__global__ void __launch_bounds__(64) k_final_verdict(const fp12 *part, const int32_t *err,
                                                      uint32_t nparts, uint32_t nseg,
                                                      int32_t *verdict) {
  W12_SHARED uint32_t f[W12_WORDS], F[W12_WORDS], A[W12_WORDS], B[W12_WORDS], T[W12_WORDS],
      X[W12_WORDS], ws[W12_WS_WORDS];
  __shared__ int bad;
  int lane = threadIdx.x;
  w12_plan pl;
  w12_begin(pl, ws);
  w12_cplan cp;
  w12_cplan_load(cp, lane);
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
  // easy part: F = (conj(f) f^-1)^(p^2+1)
  w12_inv(X, f);
  w12_conj(A, f);
  w12_mul(pl, A, A, X, ws);
  w12_frob2(F, A);
  w12_mul(pl, F, F, A, ws);
  // A = F^(x-1) = F^x conj(F);  A = A^(x-1)
  w12_cyc_exp_x(pl, cp, A, F, ws);
  w12_conj(X, F);
  w12_mul(pl, A, A, X, ws);
  w12_cyc_exp_x(pl, cp, B, A, ws);
  w12_conj(X, A);
  w12_mul(pl, A, B, X, ws);
  // B = A^(x+p) = A^x frob(A)
  w12_cyc_exp_x(pl, cp, B, A, ws);
  w12_frob(X, A);
  w12_mul(pl, B, B, X, ws);
  // T = B^x;  C = T^x frob2(B) conj(B)   (C in A)
  w12_cyc_exp_x(pl, cp, T, B, ws);
  w12_cyc_exp_x(pl, cp, A, T, ws);
  w12_frob2(X, B);
  w12_mul(pl, A, A, X, ws);
  w12_conj(X, B);
  w12_mul(pl, A, A, X, ws);
  // R = C F^3
  w12_mul(pl, X, F, F, ws);
  w12_mul(pl, X, X, F, ws);
  w12_mul(pl, A, A, X, ws);
  if (lane == 0) verdict[s] = (!bad && w12_is_one_image(A)) ? ST_SUCCESS : ST_VERIFY_FAIL;
}

void launch_final_verdict(hipStream_t st, const fp12 *partials, const int32_t *err,
                          uint32_t nparts, uint32_t nseg, int32_t *verdict) {
  if (nseg) k_final_verdict<<<nseg, 64, 0, st>>>(partials, err, nparts, nseg, verdict);
}

}  // namespace gbls
