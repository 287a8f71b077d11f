// gfx950 kernels: hash_to_G2 (a13, RFC 9380 BLS12381G2_XMD:SHA-256_SSWU_RO_ with the
// Ethereum POP DST, bls/src/consts.rs:1) stage 1 (expand_message_xmd + hash_to_field), one lane per message (or
// per field element for the SSWU map).  Output: affine points (Miller-loop input).
#include "gbls_common.h"

namespace gbls {

__device__ __constant__ uint8_t DST_POP[43] = {
    'B', 'L', 'S', '_', 'S', 'I', 'G', '_', 'B', 'L', 'S', '1', '2', '3', '8', '1',
    'G', '2', '_', 'X', 'M', 'D', ':', 'S', 'H', 'A', '-', '2', '5', '6', '_', 'S',
    'S', 'W', 'U', '_', 'R', 'O', '_', 'P', 'O', 'P', '_'};

// stage 1: expand_message_xmd + hash_to_field -> u[0], u[1].  off == nullptr: 32-byte
// messages packed back to back (signing roots, verifier.rs:307).
__global__ void __launch_bounds__(WG) k_h2c_field(const uint8_t *msg, const uint32_t *off,
                                                  uint32_t n, const uint8_t *dst, uint32_t dlen,
                                                  fp2 *U) {
  uint32_t i = blockIdx.x * WG + threadIdx.x;
  if (i >= n) return;
  const uint8_t *p;
  uint32_t len;
  if (off) {
    p = msg + off[i];
    len = off[i + 1] - off[i];
  } else {
    p = msg + 32u * i;
    len = 32;
  }
  fp2 u[2];
  hash_to_field_g2(u, p, len, dst_ref{dst ? dst : DST_POP, dst ? dlen : 43u});
  U[2 * i] = u[0];
  U[2 * i + 1] = u[1];
}
void launch_h2c_field(hipStream_t st, const uint8_t *msg, const uint32_t *off, uint32_t n,
                      const uint8_t *dst, uint32_t dlen, fp2 *U) {
  if (n) k_h2c_field<<<nblk(n), WG, 0, st>>>(msg, off, n, dst, dlen, U);
}
}  // namespace gbls
