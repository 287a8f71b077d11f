// gfx950 kernels: hash_to_G2 (a13, RFC 9380 BLS12381G2_XMD:SHA-256_SSWU_RO_ with the
// Ethereum POP DST, bls/src/consts.rs:1) stage 2 (SSWU map to E2' + 3-isogeny), one lane per message (or
// per field element for the SSWU map).  Output: affine points (Miller-loop input).
#include "gbls_common.h"

namespace gbls {

// stage 2: one lane per field element: SSWU on E2' + 3-isogeny -> Jacobian on E2
__global__ void __launch_bounds__(WG) k_h2c_map(const fp2 *U, uint32_t nu, g2j *Q) {
  uint32_t i = blockIdx.x * WG + threadIdx.x;
  if (i >= nu) return;
  g2j q;
  map_to_g2(q, U[i]);
  Q[i] = q;
}
void launch_h2c_map(hipStream_t st, const fp2 *U, uint32_t nu, g2j *Q) {
  if (nu) k_h2c_map<<<nblk(nu), WG, 0, st>>>(U, nu, Q);
}
}  // namespace gbls
