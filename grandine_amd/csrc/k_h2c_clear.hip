// gfx950 kernels: hash_to_G2 (a13, RFC 9380 BLS12381G2_XMD:SHA-256_SSWU_RO_ with the
// Ethereum POP DST, bls/src/consts.rs:1) stage 3 (Q0 + Q1, cofactor clearing, affine), one lane per message (or
// per field element for the SSWU map).  Output: affine points (Miller-loop input).
#include "gbls_common.h"

namespace gbls {

// stage 3: Q0 + Q1, clear the cofactor (Budroni-Pintore), affine
__global__ void __launch_bounds__(WG) k_h2c_clear(const g2j *Q, uint32_t n, g2a *H) {
  uint32_t i = blockIdx.x * WG + threadIdx.x;
  if (i >= n) return;
  g2j a = Q[2 * i], b = Q[2 * i + 1], h;
  jac_add(a, a, b);
  clear_cofactor_g2(h, a);
  g2a o;
  jac_to_aff(o, h);
  H[i] = o;
}

void launch_h2c_clear(hipStream_t st, const g2j *Q, uint32_t n, g2a *H) {
  k_h2c_clear<<<nblk(n), WG, 0, st>>>(Q, n, H);
}

}  // namespace gbls
