// gfx950 kernel: the 68 Miller-loop line functions (63 doubling + 5 addition steps
// along |x|) of every pair's G2 point, one lane per pair, stored structure-of-arrays
// (bls_pairing.h line_word) so that each later load is one coalesced dword per lane.
#include "gbls_common.h"

namespace gbls {

__global__ void __launch_bounds__(WG) k_lines(const g2a *H, uint32_t first, uint32_t count,
                                              uint32_t np, uint32_t *L) {
  uint32_t i = blockIdx.x * WG + threadIdx.x;
  if (i >= count) return;
  g2a q = H[first + i];
  lines_of(L, np, first + i, q);
}

void launch_lines(hipStream_t st, const g2a *H, uint32_t first, uint32_t count, uint32_t np,
                  uint32_t *lines) {
  if (count) k_lines<<<nblk(count), WG, 0, st>>>(H, first, count, np, lines);
}

}  // namespace gbls
