// gfx950 kernel: the 68 Miller-loop line functions (63 doubling + 5 addition steps
// along |x|) of every pair's G2 point, stored structure-of-arrays (bls_pairing.h
// line_word) so that each later load is one coalesced dword per lane.  One DPP quad per
// pair: doubling and addition steps run quad-cooperatively (bls_gang.h gang_line_dbl,
// gang_line_add_aff); lane q stores line components c with c % 4 == q.  Large batches
// generate and consume the lines in event slices (the running point T kept in HBM
// between slices), so the buffer holds a slice of events, not all 68.  Launches of at
// least kLaneRegimeLines pairs run one pair per lane instead (k_lines_lane).
#include "gbls_common.h"
#define GBLS_GANG_LINES
#include "bls_gang.h"

namespace gbls {

__device__ __forceinline__ void line_put_q(uint32_t *L, uint32_t np, uint32_t pair, int e, int q,
                                           const fp2 &L0, const fp2 &L2, const fp2 &L3) {
  const fp *v[6] = {&L0.c0, &L0.c1, &L2.c0, &L2.c1, &L3.c0, &L3.c1};
#pragma unroll
  for (int c = 0; c < 6; c++) {
    if ((c & 3) != q) continue;
#pragma unroll
    for (int i = 0; i < 12; i++) L[line_word(e, c, i, np, pair)] = v[c]->l[i];
  }
}

__device__ __forceinline__ void line_put_row(uint32_t *L, uint32_t np, uint32_t pair, int e, int l,
                                             const fp2 &L0, const fp2 &L2, const fp2 &L3) {
  const fp *v[6] = {&L0.c0, &L0.c1, &L2.c0, &L2.c1, &L3.c0, &L3.c1};
#pragma unroll
  for (int c = 0; c < 6; c++) {
    if (c != l) continue;
#pragma unroll
    for (int i = 0; i < 12; i++) L[line_word(e, c, i, np, pair)] = v[c]->l[i];
  }
}

// lines_range (bls_pairing.h) with quad doubling and addition steps: events [e0, e1)
__global__ void __launch_bounds__(WG) k_lines(const g2a *H, uint32_t first, uint32_t count,
                                              uint32_t np, int e0, int e1, g2h *Ts, uint32_t *L) {
  uint32_t t = blockIdx.x * WG + threadIdx.x;
  uint32_t i = t >> 2;
  int q = (int)(t & 3);
  if (i >= count) return;  // whole quads only
  uint32_t pair = first + i;
  g2a Q = H[pair];
  fp2 L0, L2, L3;
  if (aff_is_inf(Q)) {
    fp2_one(L0);
    fp2_zero(L2);
    fp2_zero(L3);
    for (int e = e0; e < e1; e++) line_put_q(L, np, pair, e - e0, q, L0, L2, L3);
    return;
  }
  g2h T;
  if (e0 > 0) {
    T = Ts[pair];
  } else {
    T.x = Q.x;
    T.y = Q.y;
    fp2_one(T.z);
  }
  for (int e = e0; e < e1; e++) {
    if (ev_is_dbl(e))
      gang_line_dbl(T, L0, L2, L3, q);
    else
      gang_line_add_aff(T, Q, L0, L2, L3, q);
    line_put_q(L, np, pair, e - e0, q, L0, L2, L3);
  }
  if (e1 < ML_EVENTS && q == 0) Ts[pair] = T;
}

// the same on a 16-lane row (small launches); lanes 0-5 store one component each
__global__ void __launch_bounds__(WG) k_lines_row(const g2a *H, uint32_t first, uint32_t count,
                                                  uint32_t np, int e0, int e1, g2h *Ts,
                                                  uint32_t *L) {
  uint32_t t = blockIdx.x * WG + threadIdx.x;
  uint32_t i = t >> 4;
  int l = (int)(t & 15);
  if (i >= count) return;  // whole rows
  uint32_t pair = first + i;
  g2a Q = H[pair];
  fp2 L0, L2, L3;
  if (aff_is_inf(Q)) {
    fp2_one(L0);
    fp2_zero(L2);
    fp2_zero(L3);
    for (int e = e0; e < e1; e++) line_put_row(L, np, pair, e - e0, l, L0, L2, L3);
    return;
  }
  g2h T;
  if (e0 > 0) {
    T = Ts[pair];
  } else {
    T.x = Q.x;
    T.y = Q.y;
    fp2_one(T.z);
  }
  for (int e = e0; e < e1; e++) {
    if (ev_is_dbl(e))
      row_line_dbl(T, L0, L2, L3, l);
    else
      row_line_add_aff(T, Q, L0, L2, L3, l);
    line_put_row(L, np, pair, e - e0, l, L0, L2, L3);
  }
  if (e1 < ML_EVENTS && l == 0) Ts[pair] = T;
}

// one lane per pair (serial lines_range): a quarter of the quad's instructions per pair,
// for launches that fill the chip on their own
__global__ void __launch_bounds__(WG) k_lines_lane(const g2a *H, uint32_t first, uint32_t count,
                                                   uint32_t np, int e0, int e1, g2h *Ts,
                                                   uint32_t *L) {
  uint32_t i = blockIdx.x * WG + threadIdx.x;
  if (i >= count) return;
  g2a Q = H[first + i];
  lines_range(L, np, first + i, Q, e0, e1, Ts);
}

void launch_lines(hipStream_t st, const g2a *H, uint32_t first, uint32_t count, uint32_t np,
                  int e0, int e1, g2h *Ts, uint32_t *lines) {
  if (!count) return;
  if (count >= kLaneRegimeLines)
    k_lines_lane<<<nblk(count), WG, 0, st>>>(H, first, count, np, e0, e1, Ts, lines);
  else if (count <= kRowRegimeMax)
    k_lines_row<<<nblk((size_t)count * 16), WG, 0, st>>>(H, first, count, np, e0, e1, Ts, lines);
  else
    k_lines<<<nblk((size_t)count * 4), WG, 0, st>>>(H, first, count, np, e0, e1, Ts, lines);
}

}  // namespace gbls
