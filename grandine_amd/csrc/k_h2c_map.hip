// gfx950 kernels: hash_to_G2 (a13, RFC 9380 BLS12381G2_XMD:SHA-256_SSWU_RO_ with the
// Ethereum POP DST, bls/src/consts.rs:1) stage 2 (SSWU map to E2' + 3-isogeny), one lane per message (or
// per field element for the SSWU map).  Output: affine points (Miller-loop input).
#include "gbls_common.h"
#include "bls_dfp.h"
#include "bls_w4.h"

namespace gbls {

// stage 2: one lane per field element: SSWU on E2' + 3-isogeny -> Jacobian on E2
__global__ void __launch_bounds__(WG) k_h2c_map(const fp2 *U, uint32_t nu, g2j *Q) {
  uint32_t i = blockIdx.x * WG + threadIdx.x;
  if (i >= nu) return;
  g2j q;
  map_to_g2(q, U[i]);
  Q[i] = q;
}
// The two (p-3)/4 exponentiations of a map on the element's 16-lane row (bls_dfp.h): every
// lane of the row runs the per-lane map code redundantly on the same data, and the
// exponentiations -- 2 x 458 dependent products, most of the map's latency -- run
// row-distributed, ~2.5x faster per product than one lane's.
struct RowPow {
  __device__ void operator()(fp &r, const fp &a) const {
    dfp::Tabs t;
    dfp::load_tabs(t);
#if defined(GBLS_MAP_NOPOW)  // timing experiment (wrong points)
    const uint32_t x = dfp::from_regs(a.l, t);
#else
    const uint32_t x = dfp::pow_pm3d4(dfp::from_regs(a.l, t), t);
#endif
    dfp::to_words_all(r.l, x, t);
  }
};
template <bool X>
__global__ void __launch_bounds__(WG) k_h2c_map_row(const fp2 *U, uint32_t nu, g2j *Q) {
  if constexpr (X) w4::exclusive_simd();
  const uint32_t i = (blockIdx.x * WG + threadIdx.x) >> 4;
  if (i >= nu) return;  // whole rows
  g2j q;
  map_to_g2(q, U[i], RowPow());
  if ((threadIdx.x & 15) == 0) Q[i] = q;
}

// field elements up to g_map_rows_max (2048 unless GBLS_MAP_ROWS_MAX is set) take the row form
// (16 lanes each: 512 waves at 2048)

void launch_h2c_map(hipStream_t st, const fp2 *U, uint32_t nu, g2j *Q) {
  if (!nu) return;
  if (nu <= g_map_rows_max)
    (nblk((size_t)nu * 16) <= w4::kExclusiveMaxWaves ? k_h2c_map_row<true> : k_h2c_map_row<false>)<<<
        nblk((size_t)nu * 16), WG, 0, st>>>(U, nu, Q);
  else
    k_h2c_map<<<nblk(nu), WG, 0, st>>>(U, nu, Q);
}
}  // namespace gbls
