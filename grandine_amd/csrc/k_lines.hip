// gfx950 kernel: the 68 Miller-loop line functions (63 doubling + 5 addition steps
// along |x|) of every pair's G2 point, stored structure-of-arrays (bls_pairing.h
// line_word) so that each later load is one coalesced dword per lane.  A pair's lines go to
// its COLUMN (LineCols: col[pair], or the pair itself): the Miller-product tables place pair
// j of group g at column j ngp + g (ngp = groups rounded up to 64), so that every wave of
// k_ml_group reads 64 consecutive, 256-byte-aligned words per load (r05: the pair-indexed
// layout straddled three 128-B lines per wave load, 1.38x the line bytes in FETCH_SIZE).  One DPP quad per
// pair: doubling and addition steps run quad-cooperatively (bls_gang.h gang_line_dbl,
// gang_line_add_aff); lane q stores line components c with c % 4 == q.  Large batches
// generate and consume the lines in event slices (the running point T kept in HBM
// between slices), so the buffer holds a slice of events, not all 68.  Launches of at
// least g_lane_min pairs run one pair per lane instead (k_lines_lane).
#include "gbls_common.h"
#define GBLS_GANG_LINES
#include "bls_gang.h"
#include "bls_w4.h"
#include "bls_curve28.h"

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
                                              LineCols lc, int e0, int e1, g2h *Ts, uint32_t *L) {
  uint32_t t = blockIdx.x * WG + threadIdx.x;
  uint32_t i = t >> 2;
  int q = (int)(t & 3);
  if (i >= count) return;  // whole quads only
  uint32_t pair = first + i;
  const uint32_t np = lc.ncol, cp = lc.col ? lc.col[pair] : pair;  // the line column
  g2a Q = H[pair];
  fp2 L0, L2, L3;
  if (aff_is_inf(Q)) {
    fp2_one(L0);
    fp2_zero(L2);
    fp2_zero(L3);
    for (int e = e0; e < e1; e++) line_put_q(L, np, cp, e - e0, q, L0, L2, L3);
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
    line_put_q(L, np, cp, e - e0, q, L0, L2, L3);
  }
  if (e1 < ML_EVENTS && q == 0) Ts[pair] = T;
}

// the same on a 16-lane row (small launches); lanes 0-5 store one component each
__global__ void __launch_bounds__(WG) k_lines_row(const g2a *H, uint32_t first, uint32_t count,
                                                  LineCols lc, int e0, int e1, g2h *Ts,
                                                  uint32_t *L) {
  uint32_t t = blockIdx.x * WG + threadIdx.x;
  uint32_t i = t >> 4;
  int l = (int)(t & 15);
  if (i >= count) return;  // whole rows
  uint32_t pair = first + i;
  const uint32_t np = lc.ncol, cp = lc.col ? lc.col[pair] : pair;  // the line column
  g2a Q = H[pair];
  fp2 L0, L2, L3;
  if (aff_is_inf(Q)) {
    fp2_one(L0);
    fp2_zero(L2);
    fp2_zero(L3);
    for (int e = e0; e < e1; e++) line_put_row(L, np, cp, e - e0, l, L0, L2, L3);
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
    line_put_row(L, np, cp, e - e0, l, L0, L2, L3);
  }
  if (e1 < ML_EVENTS && l == 0) Ts[pair] = T;
}

// The lane regime's line steps (bls_pairing.h line_dbl / line_add_aff, the same operations on
// the same operands, so the same values) reordered so that each line coefficient is stored as
// soon as it is known: the three Fp2 coefficients (72 registers) are never live together with
// the step's temporaries, which kept k_lines_lane spilling 196 B per lane.
__device__ __forceinline__ void put_fp2(uint32_t *L, uint32_t np, uint32_t pair, int e, int c, const fp2 &v) {
#pragma unroll
  for (int i = 0; i < 12; i++) L[line_word(e, c, i, np, pair)] = v.c0.l[i];
#pragma unroll
  for (int i = 0; i < 12; i++) L[line_word(e, c + 1, i, np, pair)] = v.c1.l[i];
}
__device__ __forceinline__ void lane_line_dbl(g2h &T, uint32_t *L, uint32_t np, uint32_t pair, int e) {
  fp2 A, B, E, H, t;
  fp2_sqr(B, T.y);       // Y^2
  fp2_sqr(t, T.z);       // C = Z^2
  fp2_mul_3b(E, t);      // 3b'Z^2
  fp2_add(H, T.y, T.z);
  fp2_sqr(H, H);
  fp2_sub(H, H, B);
  fp2_sub(H, H, t);      // 2YZ                      (C dead)
  fp2_mul(A, T.x, T.y);
  fp2_half(A, A);        // XY/2                     (Y dead)
  fp2_neg(t, H);
  put_fp2(L, np, pair, e, 4, t);  // L3 = -2YZ
  fp2_sub(t, E, B);
  put_fp2(L, np, pair, e, 0, t);  // L0 = 3b'Z^2 - Y^2
  fp2_sqr(t, T.x);
  fp2_mul3(t, t);
  put_fp2(L, np, pair, e, 2, t);  // L2 = 3X^2          (X dead)
  fp2 F;
  fp2_add(F, E, E);
  fp2_add(F, F, E);      // 3E
  fp2_sub(t, B, F);
  fp2_mul(T.x, A, t);    // X3 = A (B - F)          (A dead)
  fp2_mul(T.z, B, H);    // Z3 = B H                (H dead)
  fp2_add(t, B, F);
  fp2_half(t, t);
  fp2_sqr(t, t);         // G^2
  fp2_sqr(E, E);
  fp2_mul3(E, E);        // 3E^2
  fp2_sub(T.y, t, E);    // Y3 = G^2 - 3E^2
}
__device__ __forceinline__ void lane_line_add_aff(g2h &T, const g2a &Q, uint32_t *L, uint32_t np, uint32_t pair,
                                                  int e) {
  fp2 th, la, t, u;
  fp2_mul(t, Q.y, T.z);
  fp2_sub(th, T.y, t);
  fp2_mul(t, Q.x, T.z);
  fp2_sub(la, T.x, t);
  fp2_mul(u, th, Q.x);
  fp2_mul(t, la, Q.y);
  fp2_sub(u, u, t);
  put_fp2(L, np, pair, e, 0, u);   // L0 = theta x2 - lambda y2
  fp2_neg(u, th);
  put_fp2(L, np, pair, e, 2, u);   // L2 = -theta
  put_fp2(L, np, pair, e, 4, la);  // L3 = lambda
  fp2 vv, vvv, R, A;
  fp2_sqr(u, th);                  // uu
  fp2_sqr(vv, la);
  fp2_mul(vvv, vv, la);
  fp2_neg(vvv, vvv);       // v^3 = -lambda^3
  fp2_mul(R, vv, T.x);
  fp2_mul(A, u, T.z);
  fp2_sub(A, A, vvv);
  fp2_sub(A, A, R);
  fp2_sub(A, A, R);
  fp2_mul(T.x, la, A);
  fp2_neg(T.x, T.x);       // X3 = v A
  fp2_sub(t, R, A);
  fp2_mul(t, th, t);
  fp2_neg(t, t);           // u (R - A)
  fp2_mul(R, vvv, T.y);
  fp2_sub(T.y, t, R);
  fp2_mul(T.z, vvv, T.z);
}

// one lane per pair (serial lines_range): a quarter of the quad's instructions per pair,
// for launches that fill the chip on their own
__global__ void __launch_bounds__(WG) k_lines_lane(const g2a *H, uint32_t first, uint32_t count,
                                                   LineCols lc, int e0, int e1, g2h *Ts,
                                                   uint32_t *L) {
  uint32_t i = blockIdx.x * WG + threadIdx.x;
  if (i >= count) return;
  const uint32_t pair = first + i;
  const uint32_t np = lc.ncol, cp = lc.col ? lc.col[pair] : pair;  // the line column
  const g2a Q = H[pair];
  if (aff_is_inf(Q)) {
    lines_range(L, np, cp, Q, e0, e1, Ts);  // identity lines
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
      lane_line_dbl(T, L, np, cp, e - e0);
    else
      lane_line_add_aff(T, Q, L, np, cp, e - e0);
  }
  if (e1 < ML_EVENTS) Ts[pair] = T;
}

// The lane regime in radix 2^28 (bls_curve28.h line_dbl28 / line_add28: one v_mad_u64_u32 per
// product term instead of a mad + carry pair), the default since r05 (g_lane_r28).  Q (affine,
// engine form) is converted once; T runs in radix 2^28; every coefficient is stored as its
// repacked limbs (store12: no conversion product), which an engine-form reader sees as the
// coefficient times 2^8 -- one scalar for the whole line, removed by the final exponentiation
// (as the W4 form's 2^64).  Q's coordinates wait in LDS for the 5 addition steps; between the
// event slices of a sliced submission T is stored in engine form, as every other form does.
__device__ __forceinline__ void put28(uint32_t *L, uint32_t np, uint32_t pair, int e, int c, const r28::fe2 &v) {
  fp w;
  r28::store12(w, v.c0);
#pragma unroll
  for (int i = 0; i < 12; i++) L[line_word(e, c, i, np, pair)] = w.l[i];
  r28::store12(w, v.c1);
#pragma unroll
  for (int i = 0; i < 12; i++) L[line_word(e, c + 1, i, np, pair)] = w.l[i];
}
__global__ void __launch_bounds__(WG) k_lines_lane28(const g2a *H, uint32_t first, uint32_t count,
                                                     LineCols lc, int e0, int e1, g2h *Ts, uint32_t *L) {
  uint32_t i = blockIdx.x * WG + threadIdx.x;
  if (i >= count) return;
  const uint32_t pair = first + i;
  const uint32_t np = lc.ncol, cp = lc.col ? lc.col[pair] : pair;  // the line column
  const g2a Q = H[pair];
  if (aff_is_inf(Q)) {
    lines_range(L, np, cp, Q, e0, e1, Ts);  // identity lines (engine form)
    return;
  }
  // Q's coordinates in LDS at an odd stride of 29 words per lane (28 + 1 pad): conflict-free
  // 4-byte accesses (the unpadded 28-word stride put every 8th lane of a group on one bank)
  struct fe2_lds {
    r28::fe2 v;
    uint32_t pad;
  };
  static_assert(sizeof(fe2_lds) == 29 * 4, "odd LDS stride");
  __shared__ fe2_lds qs[2 * WG];
  r28::fe2 &qx = qs[threadIdx.x].v, &qy = qs[WG + threadIdx.x].v;
  r28::g2h28 T;
  r28::from_fp(T.x.c0, Q.x.c0);
  r28::from_fp(T.x.c1, Q.x.c1);
  r28::from_fp(T.y.c0, Q.y.c0);
  r28::from_fp(T.y.c1, Q.y.c1);
  qx = T.x;
  qy = T.y;
  if (e0 > 0) {  // T between slices is engine form whatever kernel form wrote it
    const g2h &t = Ts[pair];
    r28::from_fp(T.x.c0, t.x.c0), r28::from_fp(T.x.c1, t.x.c1);
    r28::from_fp(T.y.c0, t.y.c0), r28::from_fp(T.y.c1, t.y.c1);
    r28::from_fp(T.z.c0, t.z.c0), r28::from_fp(T.z.c1, t.z.c1);
  } else {
    r28::f_one(T.z);
  }
  for (int e = e0; e < e1; e++) {
    const int el = e - e0;
    auto put = [&](int c, const r28::fe2 &v) { put28(L, np, cp, el, c, v); };
    if (ev_is_dbl(e))
      r28::line_dbl28(T, put);
    else
      r28::line_add28(T, qx, qy, put);
  }
  if (e1 < ML_EVENTS) {
    g2h &t = Ts[pair];
    r28::to_fp(t.x.c0, T.x.c0), r28::to_fp(t.x.c1, T.x.c1);
    r28::to_fp(t.y.c0, T.y.c0), r28::to_fp(t.y.c1, T.y.c1);
    r28::to_fp(t.z.c0, T.z.c0), r28::to_fp(t.z.c1, T.z.c1);
  }
}

// one wave per pair (bls_w4.h), the smallest launches: a doubling step is six rounds of four
// row-distributed products, the six line words two more (canonical engine form, SoA as above)
__device__ __forceinline__ void line_put_w4(const w4::Ctx &c, uint32_t *L, uint32_t np, uint32_t pair,
                                            int e, const w4::f2 &l0, const w4::f2 &l2, const w4::f2 &l3) {
  // the coefficients times 2^64 (dfp::word_of_scaled: no conversion product; an Fp* factor per
  // line, which the final exponentiation removes)
  const uint32_t j = c.t.j;
  uint32_t w = dfp::word_of_scaled(w4::sel(c, l0.c0, l0.c1, l2.c0, l2.c1));
  if (j < 12) L[line_word(e, (int)c.r, (int)j, np, pair)] = w;
  w = dfp::word_of_scaled(w4::sel(c, l3.c0, l3.c1, l3.c0, l3.c1));
  if (j < 12 && c.r < 2) L[line_word(e, 4 + (int)c.r, (int)j, np, pair)] = w;
}
template <bool X>
__global__ void __launch_bounds__(64) k_lines_w4(const g2a *H, uint32_t first, uint32_t count,
                                                 LineCols lc, int e0, int e1, g2h *Ts, uint32_t *L) {
  if constexpr (X) w4::exclusive_simd();
  const uint32_t i = blockIdx.x;
  if (i >= count) return;  // whole waves
  const uint32_t pair = first + i;
  const uint32_t np = lc.ncol, cp = lc.col ? lc.col[pair] : pair;  // the line column
  const g2a Q = H[pair];
  const uint32_t j = threadIdx.x & 15, r = (threadIdx.x >> 4) & 3;
  if (aff_is_inf(Q)) {  // identity lines: L0 = 1, L2 = L3 = 0
    uint32_t one = 0;
#pragma unroll
    for (int k = 0; k < 12; k++) one = j == (uint32_t)k ? k::ONE_M[k] : one;
    for (int e = e0; e < e1; e++)
      for (uint32_t cc = r; cc < 6; cc += 4)
        if (j < 12) L[line_word(e - e0, (int)cc, (int)j, np, cp)] = cc == 0 ? one : 0u;
    return;
  }
  w4::Ctx c;
  w4::init(c);
  w4::A2 q;
  w4::load(c, q, Q);
  w4::J T;
  if (e0 > 0) {
    g2j tj;
    tj.x = Ts[pair].x;
    tj.y = Ts[pair].y;
    tj.z = Ts[pair].z;
    w4::load(c, T, tj);
  } else {
    T.x = q.x;
    T.y = q.y;
    T.z = {c.one, 0u};
  }
  for (int e = e0; e < e1; e++) {
    w4::f2 l0, l2, l3;
    if (ev_is_dbl(e))
      w4::line_dbl(c, T, l0, l2, l3);
    else
      w4::line_add_aff(c, T, q, l0, l2, l3);
    line_put_w4(c, L, np, cp, e - e0, l0, l2, l3);
  }
  if (e1 < ML_EVENTS) {
    g2h *o = Ts + pair;
    w4::store4(c, T.x.c0, T.x.c1, T.y.c0, T.y.c1, o->x.c0.l, o->x.c1.l, o->y.c0.l, o->y.c1.l);
    uint32_t w = dfp::word_of(w4::sel(c, T.z.c0, T.z.c1, T.z.c0, T.z.c1), c.t);
    if (j < 12 && r == 0) o->z.c0.l[j] = w;
    if (j < 12 && r == 1) o->z.c1.l[j] = w;
  }
}

// all 68 events of pairs [0, count) from Jacobian points Qj[stride i] (k_h2c_clear_w4j):
// T starts as the homogeneous form of Q and the addition steps take Q projectively (lines
// scaled by Fp2 factors, which the final exponentiation removes)
template <bool X>
__global__ void __launch_bounds__(64) k_lines_w4j(const g2j *Qj, uint32_t stride, uint32_t first,
                                                  uint32_t count, LineCols lc, uint32_t *L) {
  if constexpr (X) w4::exclusive_simd();
  const uint32_t i = blockIdx.x, pair = first + i;
  if (i >= count) return;  // whole waves
  const uint32_t np = lc.ncol, cp = lc.col ? lc.col[pair] : pair;  // the line column
  const uint32_t j = threadIdx.x & 15, r = (threadIdx.x >> 4) & 3;
  w4::Ctx c;
  w4::init(c);
  w4::J q;
  w4::load(c, q, Qj[(size_t)stride * i]);
  if (w4::is_inf(c, q)) {  // identity lines: L0 = 1, L2 = L3 = 0
    uint32_t one = 0;
#pragma unroll
    for (int k = 0; k < 12; k++) one = j == (uint32_t)k ? k::ONE_M[k] : one;
    for (int e = 0; e < ML_EVENTS; e++)
      for (uint32_t cc = r; cc < 6; cc += 4)
        if (j < 12) L[line_word(e, (int)cc, (int)j, np, cp)] = cc == 0 ? one : 0u;
    return;
  }
  w4::jac_to_hom(c, q, q);
  w4::J T = q;
  for (int e = 0; e < ML_EVENTS; e++) {
    w4::f2 l0, l2, l3;
    if (ev_is_dbl(e))
      w4::line_dbl(c, T, l0, l2, l3);
    else
      w4::line_add_proj(c, T, q, l0, l2, l3);
    line_put_w4(c, L, np, cp, e, l0, l2, l3);
  }
}
bool launch_lines_jac(hipStream_t st, const g2j *Qj, uint32_t stride, uint32_t first, uint32_t count,
                      LineCols lc, uint32_t *lines) {
  if (!count || count > kW4Max) return false;
  (count <= w4::kExclusiveMaxWaves ? k_lines_w4j<true> : k_lines_w4j<false>)<<<count, 64, 0, st>>>(
      Qj, stride, first, count, lc, lines);
  return true;
}

void launch_lines(hipStream_t st, const g2a *H, uint32_t first, uint32_t count, LineCols lc,
                  int e0, int e1, g2h *Ts, uint32_t *lines, bool lane) {
  if (!count) return;
  if (lane && g_lane_r28) {  // the caller asks for the one-lane form (fewest instructions per pair)
    k_lines_lane28<<<nblk(count), WG, 0, st>>>(H, first, count, lc, e0, e1, Ts, lines);
    return;
  }
  if (count <= kW4Max)
    (count <= w4::kExclusiveMaxWaves ? k_lines_w4<true> : k_lines_w4<false>)<<<count, 64, 0, st>>>(
        H, first, count, lc, e0, e1, Ts, lines);
  else if (count >= g_lane_min && g_lane_r28)
    k_lines_lane28<<<nblk(count), WG, 0, st>>>(H, first, count, lc, e0, e1, Ts, lines);
  else if (count >= g_lane_min)
    k_lines_lane<<<nblk(count), WG, 0, st>>>(H, first, count, lc, e0, e1, Ts, lines);
  else if (count <= kRowRegimeMax)
    k_lines_row<<<nblk((size_t)count * 16), WG, 0, st>>>(H, first, count, lc, e0, e1, Ts, lines);
  else
    k_lines<<<nblk((size_t)count * 4), WG, 0, st>>>(H, first, count, lc, e0, e1, Ts, lines);
}

}  // namespace gbls
