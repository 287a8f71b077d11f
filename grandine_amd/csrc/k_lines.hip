// gfx950 kernel: the 68 Miller-loop line functions (63 doubling + 5 addition steps
// along |x|) of every pair's G2 point, one lane per pair, stored structure-of-arrays
// (bls_pairing.h line_word) so that each later load is one coalesced dword per lane.
#include "gbls_common.h"

namespace gbls {

__global__ void __launch_bounds__(WG) k_lines(const g2a *H, uint32_t np, uint32_t *L) {
  uint32_t i = blockIdx.x * WG + threadIdx.x;
  if (i >= np) return;
  g2a q = H[i];
  lines_of(L, np, i, q);
}

void launch_lines(hipStream_t st, const g2a *H, uint32_t np, uint32_t *lines) {
  k_lines<<<nblk(np), WG, 0, st>>>(H, np, lines);
}

}  // namespace gbls
