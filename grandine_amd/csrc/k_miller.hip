// gfx950 kernels: the batch Miller product as a tree (bls_pairing.h header comment).
//   k_ml_group  lane per (event e, group of <= G pairs of one segment): the product of
//               the group's evaluated lines, line_e(P_a) line_e(P_b) ... (sparse x sparse,
//               then dense x sparse), in registers -> one dense Fp12.  A group's pairs are
//               strided through its segment's pair list (pair k, k + ng, k + 2 ng, ...
//               for ng groups), so lanes of a wave load the SoA line words of adjacent
//               pairs: coalesced.  G grows with the batch (bigger G = fewer values for
//               the wave-cooperative levels, which are 3x less efficient per product).
//   k_ml_reduce wave per (event, group of <= 4 values of one segment): wave-cooperative
//               Fp12 products (bls_wave12.h)
//   k_ml_horner wave per segment: Horner over the 68 events, then conj (x < 0)
#include "bls_wave12.h"
#include "bls_w12d.h"
#include "bls_field28.h"
#include "gbls_common.h"

namespace gbls {

// the line column of pair j of group g (pair id `pair`): the tables' layout j ngp + g, or lc's
__device__ __forceinline__ uint32_t ml_col(const LineCols &lc, uint32_t ngp, uint32_t g, uint32_t j,
                                           uint32_t pair) {
  return ngp ? j * ngp + g : (lc.col ? lc.col[pair] : pair);
}
__device__ __forceinline__ void ml_eval(sp034 &s, const uint32_t *L, uint32_t ncol, uint32_t col,
                                        const g1s *P, uint32_t pair, int e) {
  fp2 L0, L2, L3;
  line_get(L, ncol, col, e, L0, L2, L3);
  g1s Pp = P[pair];
  line_eval_s(s, L0, L2, L3, Pp);
}

// One block per (group block gb of 64 groups, event el): nbx * ne blocks in a 1-D grid.  XCD
// order (g_ml_xcd): the dispatcher deals blocks round-robin over the 8 XCDs (MI355X_MICROARCH
// "Workgroup dispatch"), so block b's work index is remapped (bijectively) to give each XCD a
// contiguous run of work with the event fastest: the ne blocks of a group block run together
// on ONE XCD and read its pairs' G1 points from that XCD's L2 once, instead of every event
// re-reading them from HBM (the r04 launch fetched 2.33 GB for 1.35 GB of lines).  Group g =
// (first plist index, stride, count); the lines buffer holds events [e0, e0 + ne) at e - e0.
__device__ __forceinline__ uint32_t xcd_work_index(uint32_t b, uint32_t nwg) {
  const uint32_t xcd = b % 8, q = nwg / 8, r = nwg % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + b / 8;
}
__global__ void __launch_bounds__(WG) k_ml_group(const uint32_t *L, LineCols lc, uint32_t ngp, const g1s *P,
                                                 const uint32_t *plist, const uint32_t *grp,
                                                 uint32_t ngroup, int e0, int ne, int xcd_order,
                                                 fp12 *V0) {
  const uint32_t nwg = gridDim.x;
  uint32_t w = blockIdx.x, gb;
  int el;
  if (xcd_order) {
    w = xcd_work_index(w, nwg);
    gb = w / (uint32_t)ne;
    el = (int)(w % (uint32_t)ne);
  } else {  // the r04 order: event-major
    gb = w % (nwg / (uint32_t)ne);
    el = (int)(w / (nwg / (uint32_t)ne));
  }
  uint32_t g = gb * WG + threadIdx.x;
  int e = e0 + el;
  if (g >= ngroup) return;
  uint32_t at = grp[3 * g], stride = grp[3 * g + 1], cnt = grp[3 * g + 2];
  const uint32_t nc = lc.ncol;
  auto eval = [&](sp034 &sx, uint32_t j) {
    const uint32_t pair = plist[at + j * stride];
    ml_eval(sx, L, nc, ml_col(lc, ngp, g, j, pair), P, pair, el);
  };
  sp034 sa, sb;
  fp12 acc;
  eval(sa, 0);
  if (cnt == 1) {
    sp_to_fp12(acc, sa);
  } else {
    eval(sb, 1);
    sp_mul_sp(acc, sa, sb);
    for (uint32_t j = 2; j < cnt; j++) {
      eval(sa, j);
      fp12_mul_034(acc, acc, sa);
    }
  }
  V0[(size_t)e * ngroup + g] = acc;
}

// k_ml_group in radix-2^28 arithmetic (bls_field28.h), the default since r05: same grid and
// inputs; the sparse products reduce ONCE per output Fp coordinate (fe12_mul_034_lazy: six
// products per reduction, one v_mad_u64_u32 per term, no carry words), and the output differs
// from the 32-bit kernel's by an Fp scalar (2^-16 per line and 2^8 from the engine-form reading),
// which the final exponentiation removes.  g_ml_r28 = 0 (GBLS_ML_R28=0) runs the r04 kernel.
// Registers: f (168) + the line (84) + three negated line operands; the three outputs the
// in-place order parks live in LDS (fe12_mul_034_lazy_st, 84 words per lane), the line is
// evaluated one component at a time (ml_eval28), and the result leaves as raw radix-2^28
// words (k_ml_pack28 converts them): 256 VGPRs + ~140 AGPRs, no scratch.
// the line of event e at pair `pair` (line column col), evaluated at its G1 point, in radix
// 2^28: one line component (12 engine words) at a time, the next one's loads in flight during
// this one's product, so at most two components and the point's current coordinate are live.
// The point comes from Pc (the points by line column, word w of column c at w * np + c:
// coalesced, k_ml_pcols) when given, else from P; its x is loaded one component ahead of its
// use, its y two.
__device__ __forceinline__ void ml_pword(fp &r, const g1s *P, const uint32_t *Pc, uint32_t np,
                                         uint32_t col, uint32_t pair, int k) {
  if (Pc) {
#pragma unroll
    for (int i = 0; i < 12; i++) r.l[i] = Pc[(size_t)(12 * k + i) * np + col];
  } else {
    const uint32_t *w = reinterpret_cast<const uint32_t *>(P + pair) + 12 * k;
#pragma unroll
    for (int i = 0; i < 12; i++) r.l[i] = w[i];
  }
}
// The points by line column (Pc, k_ml_pcols) are NORMALIZED since r06: (x, y, c) = (2^8 xP,
// 2^8 yP, 1) for P = (xP, yP), all zero for infinity.  A line (L0 c + L2 x w^2 + L3 y w^3) then
// needs 4 products instead of 6: a0 is L0 itself, read as radix-2^28 limbs (L0 2^-8 in that
// reading), and L2 x, L3 y over 2^392 carry the same 2^-8 (the point's 2^8 cancels one of the two
// 2^-8 of the reading): one Fp* scalar per line, which the final exponentiation removes.  The
// infinity test reads one word of c (the Montgomery one's low word is nonzero).
__device__ __forceinline__ bool ml_pc_inf(const uint32_t *Pc, uint32_t np, uint32_t col) {
  return Pc[(size_t)24 * np + col] == 0;
}
template <bool PCN>
__device__ __forceinline__ void ml_eval28(r28::sp &s, const uint32_t *L, uint32_t np, uint32_t col,
                                          const g1s *P, const uint32_t *Pc, uint32_t pair, int e) {
  if constexpr (PCN) {  // normalized point: a0 = L0 read directly, 4 products
    if (ml_pc_inf(Pc, np, col)) {
      r28::sp_identity(s);
      return;
    }
    r28::fe *out[6] = {&s.a0.c0, &s.a0.c1, &s.a2.c0, &s.a2.c1, &s.a3.c0, &s.a3.c1};
    fp w, pxy;
    ml_pword(pxy, P, Pc, np, col, pair, 0);  // x, for L2
    r28::fe q;
#pragma unroll
    for (int c = 0; c < 6; c++) {
#pragma unroll
      for (int i = 0; i < 12; i++) w.l[i] = L[line_word(e, c, i, np, col)];
      if (c == 2) r28::repack_in(q, pxy);
      if (c == 2) ml_pword(pxy, P, Pc, np, col, pair, 1);  // y, for L3
      if (c == 4) r28::repack_in(q, pxy);
      asm volatile("" ::: "memory");
      if (c < 2) {
        r28::repack_in(*out[c], w);
      } else {
        r28::fe t;
        r28::repack_in(t, w);
        r28::mul(*out[c], t, q);
      }
      asm volatile("" ::: "memory");
    }
    return;
  }
  fp pc;
  ml_pword(pc, P, Pc, np, col, pair, 2);
  if (fp_is_zero(pc)) {
    r28::sp_identity(s);
    return;
  }
  r28::fe *out[6] = {&s.a0.c0, &s.a0.c1, &s.a2.c0, &s.a2.c1, &s.a3.c0, &s.a3.c1};
  uint32_t cur[12], nxt[12];
#pragma unroll
  for (int i = 0; i < 12; i++) nxt[i] = L[line_word(e, 0, i, np, col)];
  fp pxy;
  ml_pword(pxy, P, Pc, np, col, pair, 0);  // x, for L2
  r28::fe q;
  r28::repack_in(q, pc);
#pragma unroll
  for (int c = 0; c < 6; c++) {
#pragma unroll
    for (int i = 0; i < 12; i++) cur[i] = nxt[i];
    if (c < 5) {
#pragma unroll
      for (int i = 0; i < 12; i++) nxt[i] = L[line_word(e, c + 1, i, np, col)];
    }
    if (c == 2 || c == 4) r28::repack_in(q, pxy);  // the point's x for L2, its y for L3
    if (c == 2) ml_pword(pxy, P, Pc, np, col, pair, 1);
    asm volatile("" ::: "memory");
    fp w;
#pragma unroll
    for (int i = 0; i < 12; i++) w.l[i] = cur[i];
    r28::fe t;
    r28::repack_in(t, w);
    r28::mul(*out[c], t, q);
    asm volatile("" ::: "memory");
  }
}
// the line words of one pair (72, component-major) loaded as a block: the Miller kernel loads
// pair j + 1's while pair j's product runs (they wait in AGPRs), so no line load is exposed
__device__ __forceinline__ void ml_line_load(uint32_t (&lw)[72], const uint32_t *L, uint32_t np,
                                             uint32_t col, int e) {
#pragma unroll
  for (int w = 0; w < 72; w++) lw[w] = L[line_word(e, w / 12, w % 12, np, col)];
}
// ml_eval28 on a loaded line
template <bool PCN>
__device__ __forceinline__ void ml_eval28_reg(r28::sp &s, const uint32_t (&lw)[72], uint32_t np,
                                              uint32_t col, const g1s *P, const uint32_t *Pc,
                                              uint32_t pair) {
  if constexpr (PCN) {  // normalized point (see ml_eval28): a0 = L0 read directly, 4 products
    if (ml_pc_inf(Pc, np, col)) {
      r28::sp_identity(s);
      return;
    }
    r28::fe *out[6] = {&s.a0.c0, &s.a0.c1, &s.a2.c0, &s.a2.c1, &s.a3.c0, &s.a3.c1};
    fp pxy;
    ml_pword(pxy, P, Pc, np, col, pair, 0);  // x, for L2
    r28::fe q;
#pragma unroll
    for (int c = 0; c < 6; c++) {
      if (c == 2) r28::repack_in(q, pxy);
      if (c == 2) ml_pword(pxy, P, Pc, np, col, pair, 1);  // y, for L3
      if (c == 4) r28::repack_in(q, pxy);
      asm volatile("" ::: "memory");
      fp w;
#pragma unroll
      for (int i = 0; i < 12; i++) w.l[i] = lw[12 * c + i];
      if (c < 2) {
        r28::repack_in(*out[c], w);
      } else {
        r28::fe t;
        r28::repack_in(t, w);
        r28::mul(*out[c], t, q);
      }
      asm volatile("" ::: "memory");
    }
    return;
  }
  fp pc;
  ml_pword(pc, P, Pc, np, col, pair, 2);
  if (fp_is_zero(pc)) {
    r28::sp_identity(s);
    return;
  }
  r28::fe *out[6] = {&s.a0.c0, &s.a0.c1, &s.a2.c0, &s.a2.c1, &s.a3.c0, &s.a3.c1};
  fp pxy;
  ml_pword(pxy, P, Pc, np, col, pair, 0);  // x, for L2
  r28::fe q;
  r28::repack_in(q, pc);
#pragma unroll
  for (int c = 0; c < 6; c++) {
    if (c == 2 || c == 4) r28::repack_in(q, pxy);  // the point's x for L2, its y for L3
    if (c == 2) ml_pword(pxy, P, Pc, np, col, pair, 1);
    asm volatile("" ::: "memory");
    fp w;
#pragma unroll
    for (int i = 0; i < 12; i++) w.l[i] = lw[12 * c + i];
    r28::fe t;
    r28::repack_in(t, w);
    r28::mul(*out[c], t, q);
    asm volatile("" ::: "memory");
  }
}
typedef const void __attribute__((address_space(1))) *gptr_t;
typedef void __attribute__((address_space(3))) *lptr_t;
// LDS staging of the line (g_ml_dma, the default): the 72 line words of one pair's event into the wave's LDS stage (word w of lane l at
// lbuf[w * WG + l]): global -> LDS DMA loads, no VGPR destination, one coalesced dword per lane
__device__ __forceinline__ void ml_stage28(uint32_t *lbuf, const uint32_t *L, uint32_t np, uint32_t col, int e) {
#pragma unroll
  for (int w = 0; w < 72; w++)
    __builtin_amdgcn_global_load_lds((gptr_t)(L + line_word(e, w / 12, w % 12, np, col)),
                                     (lptr_t)(lbuf + w * WG), 4, 0, 0);
}
// the staged line evaluated at the pair's G1 point (loaded one pair ahead, ml_p_load), from
// the LDS words
struct MlP {
  fp x, y, c;
};
__device__ __forceinline__ void ml_p_load(MlP &p, const g1s *P, uint32_t pair) {
  const g1s *Pp = P + pair;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    p.c.l[i] = Pp->c.l[i];
    p.x.l[i] = Pp->x.l[i];
    p.y.l[i] = Pp->y.l[i];
  }
}
__device__ __forceinline__ void ml_eval28_lds(r28::sp &s, const uint32_t *lb, const MlP &p) {
  if (fp_is_zero(p.c)) {
    r28::sp_identity(s);
    return;
  }
  r28::fe *out[6] = {&s.a0.c0, &s.a0.c1, &s.a2.c0, &s.a2.c1, &s.a3.c0, &s.a3.c1};
  r28::fe q;
  r28::repack_in(q, p.c);
#pragma unroll
  for (int c = 0; c < 6; c++) {
    if (c == 2) r28::repack_in(q, p.x);
    if (c == 4) r28::repack_in(q, p.y);
    asm volatile("" ::: "memory");
    fp w;
#pragma unroll
    for (int i = 0; i < 12; i++) w.l[i] = lb[(12 * c + i) * WG];
    r28::fe t;
    r28::repack_in(t, w);
    r28::mul(*out[c], t, q);
    asm volatile("" ::: "memory");
  }
}
__device__ __forceinline__ void dma_wait() {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
}
__device__ __forceinline__ void lds_reads_done() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

template <bool DMA, bool g_prefetch, bool KARA = false, bool PCN = false>
__global__ void __launch_bounds__(WG) k_ml_group28(const uint32_t *L, LineCols lc, uint32_t ngp, const g1s *P,
                                                   const uint32_t *Pc,
                                                   const uint32_t *plist, const uint32_t *grp,
                                                   uint32_t ngroup, int e0, int ne, int xcd_order,
                                                   uint32_t *V28) {
  const uint32_t nwg = gridDim.x;
  uint32_t w = blockIdx.x, gb;
  int el;
  if (xcd_order) {
    w = xcd_work_index(w, nwg);
    gb = w / (uint32_t)ne;
    el = (int)(w % (uint32_t)ne);
  } else {
    gb = w % (nwg / (uint32_t)ne);
    el = (int)(w / (nwg / (uint32_t)ne));
  }
  uint32_t g = gb * WG + threadIdx.x;
  int e = e0 + el;
  if (g >= ngroup) return;
  uint32_t at = grp[3 * g], stride = grp[3 * g + 1], cnt = grp[3 * g + 2];
  __shared__ uint32_t park[84 * WG];
  const uint32_t np = lc.ncol;
  auto colj = [&](uint32_t j, uint32_t pair) { return ml_col(lc, ngp, g, j, pair); };
  r28::sp sa, sb;
  r28::fe12 acc;
  if constexpr (DMA) {
    // pair j + 1's line is staged into LDS by DMA loads (no VGPR destinations) while pair j's
    // product runs; the waits are vmcnt(0) + barrier before the LDS reads, lgkmcnt(0) after
    // them (the next stage overwrites the buffer)
    __shared__ uint32_t lbuf[72 * WG];
    const uint32_t *lb = lbuf + threadIdx.x;
    // the pair's G1 point is loaded with the stage (one pair ahead, into AGPRs); the next
    // pair's index right after the stage's wait, so that the evaluation hides its latency
    // (a loop-carried index load was waited at once: its VGPR -> AGPR copy)
    MlP pp;
    uint32_t pn = plist[at];
    ml_stage28(lbuf, L, np, colj(0, pn), el);
    ml_p_load(pp, P, pn);
    dma_wait();
    pn = plist[at + (cnt > 1 ? stride : 0)];  // unconditional: a phi would wait on the load
    ml_eval28_lds(sa, lb, pp);
    lds_reads_done();
    if (cnt == 1) {
      r28::sp_to_fe12(acc, sa);
    } else {
      ml_stage28(lbuf, L, np, colj(1, pn), el);
      ml_p_load(pp, P, pn);
      dma_wait();
      pn = plist[at + (cnt > 2 ? 2 * stride : 0)];
      ml_eval28_lds(sb, lb, pp);
      lds_reads_done();
      if (cnt > 2) {
        ml_stage28(lbuf, L, np, colj(2, pn), el);
        ml_p_load(pp, P, pn);
      }
      r28::sp_mul_sp_lazy(acc, sa, sb);
      for (uint32_t j = 2; j < cnt; j++) {
        dma_wait();
        pn = plist[at + (j + 1 < cnt ? (j + 1) * stride : 0)];
        ml_eval28_lds(sa, lb, pp);
        lds_reads_done();
        if (j + 1 < cnt) {
          ml_stage28(lbuf, L, np, colj(j + 1, pn), el);
          ml_p_load(pp, P, pn);
        }
        r28::fe12_mul_034_lazy_st(acc, sa, park + threadIdx.x, WG);
      }
    }
  } else {
    // pair j + 1's line loaded while pair j's product runs (g_ml_prefetch, the default), or
    // streamed component by component inside the evaluation
    uint32_t lw[72];
    uint32_t pn = plist[at], cn = colj(0, pn);
    if (g_prefetch) ml_line_load(lw, L, np, cn, el);
    auto eval = [&](r28::sp &sx, uint32_t j) {
      const uint32_t pair = pn, cj = cn;
      if (!g_prefetch) {
        ml_eval28<PCN>(sx, L, np, cj, P, Pc, pair, el);
        if (j + 1 < cnt) pn = plist[at + (j + 1) * stride], cn = colj(j + 1, pn);
        return;
      }
      ml_eval28_reg<PCN>(sx, lw, np, cj, P, Pc, pair);
      if (j + 1 < cnt) {
        pn = plist[at + (j + 1) * stride];
        cn = colj(j + 1, pn);
        asm volatile("" ::: "memory");
        ml_line_load(lw, L, np, cn, el);
      }
    };
    eval(sa, 0);
    if (cnt == 1) {
      r28::sp_to_fe12(acc, sa);
    } else {
      eval(sb, 1);
      r28::sp_mul_sp_lazy(acc, sa, sb);
      for (uint32_t j = 2; j < cnt; j++) {
        eval(sa, j);
        if constexpr (KARA)
          r28::fe12_mul_034_kara_st(acc, sa, park + threadIdx.x, WG);
        else
          r28::fe12_mul_034_lazy_st(acc, sa, park + threadIdx.x, WG);
      }
    }
  }
  // raw radix-2^28 words, structure of arrays (word q of group g at (e * 168 + q) * ngroup + g:
  // one coalesced dword per lane per store); k_ml_pack28 converts them to engine form
  const uint32_t *ww = reinterpret_cast<const uint32_t *>(&acc);
  uint32_t *o = V28 + (size_t)e * 168 * ngroup + g;
#pragma unroll
  for (int i = 0; i < 168; i++) o[(size_t)i * ngroup] = ww[i];
}

// V28 (raw words of k_ml_group28, structure of arrays) -> V0 (engine-form fp12): one lane per
// (event, coefficient, group), the group fastest so that a wave's loads of one word are 64
// consecutive dwords (the coefficient-fastest order read 14 scattered lines per lane: 5x the
// algorithmic bytes in the r05 FETCH_SIZE pass); the canonical representative (< 1.02 p), repacked
__global__ void __launch_bounds__(WG) k_ml_pack28(const uint32_t *V28, uint32_t ngroup, int e0,
                                                  uint32_t nvals, fp12 *V0) {
  const uint32_t t = blockIdx.x * WG + threadIdx.x;
  if (t >= nvals * 12) return;
  const uint32_t g = t % ngroup, r = t / ngroup, c = r % 12, e = e0 + r / 12;
  const uint32_t *src = V28 + ((size_t)e * 168 + 14 * c) * ngroup + g;
  r28::fe x;
#pragma unroll
  for (int i = 0; i < 14; i++) x.l[i] = src[(size_t)i * ngroup];
  (void)r28::sub_p_if_geq(x);
  fp o;
  r28::repack_out(o, x);
  uint32_t *dst = reinterpret_cast<uint32_t *>(V0 + (size_t)e * ngroup + g) + 12 * c;
#pragma unroll
  for (int i = 0; i < 12; i++) dst[i] = o.l[i];
}

// copy one Fp12 image global <-> LDS with all 64 lanes
__device__ __forceinline__ void w12_load(uint32_t *dst, const fp12 *src) {
  const uint32_t *s = reinterpret_cast<const uint32_t *>(src);
  for (int i = threadIdx.x; i < W12_WORDS; i += 64) dst[i] = s[i];
  __syncthreads();
}
__device__ __forceinline__ void w12_store(fp12 *dst, const uint32_t *src) {
  uint32_t *d = reinterpret_cast<uint32_t *>(dst);
  for (int i = threadIdx.x; i < W12_WORDS; i += 64) d[i] = src[i];
}

// grid (nout, 68): output q of event e = product of Vin[e][red[2q] .. red[2q]+red[2q+1])
__global__ void __launch_bounds__(64) k_ml_reduce(const fp12 *Vin, uint32_t nin, const uint32_t *red,
                                                  uint32_t nout, fp12 *Vout) {
  W12_SHARED uint32_t acc[W12_WORDS], tmp[W12_WORDS], ws[W12_WS_WORDS];
  w12_plan pl;
  w12_begin(pl, ws);
  uint32_t q = blockIdx.x;
  int e = blockIdx.y;
  uint32_t b = red[2 * q], cnt = red[2 * q + 1];
  const fp12 *src = Vin + (size_t)e * nin + b;
  w12_load(acc, src);
  for (uint32_t j = 1; j < cnt; j++) {
    w12_load(tmp, src + j);
    w12_mul(pl, acc, acc, tmp, ws);
  }
  w12_store(Vout + (size_t)e * nout + q, acc);
}

// grid nseg: V holds one value per (event, segment): V[e * nseg + s]
__global__ void __launch_bounds__(64) k_ml_horner(const fp12 *V, uint32_t nseg, fp12 *partial,
                                                  const uint32_t *lim, uint32_t base) {
  W12_SHARED uint32_t acc[W12_WORDS], tmp[W12_WORDS], ws[W12_WS_WORDS];
  uint32_t s = blockIdx.x;
  if (lim && base + s >= *lim) return;  // block-uniform
  w12_plan pl;
  w12_begin(pl, ws);
  w12_load(acc, V + s);
  for (int e = 1; e < ML_EVENTS; e++) {
    if (ev_is_dbl(e)) w12_mul(pl, acc, acc, acc, ws);
    w12_load(tmp, V + (size_t)e * nseg + s);
    w12_mul(pl, acc, acc, tmp, ws);
  }
  w12_conj(acc, acc);
  w12_store(partial + s, acc);
}

// the pairs' G1 points by line column (Pc word w of column col[pair] at w * ncol + col): the
// Miller kernels' point loads coalesce like their line loads.  Each point is NORMALIZED on the
// way (r06): g1s (x, y, c) = (xP c, yP c, c) becomes (2^8 xP, 2^8 yP, 1), i.e. x 2^8 / c and
// y 2^8 / c with one inversion per pair (safegcd, bls_inv.h; ~40 products' worth per pair against
// the 136 products per pair its 68 line evaluations save, see ml_eval28); infinity (c = 0) stays
// all zero.  The 2^8 matches the engine-form reading of the line words (ml_eval28).
template <bool NORM>
__global__ void __launch_bounds__(WG) k_ml_pcols(const g1s *P, const uint32_t *col, uint32_t np,
                                                 uint32_t ncol, uint32_t *Pc) {
  const uint32_t pair = blockIdx.x * WG + threadIdx.x;
  if (pair >= np) return;
  const uint32_t c = col[pair];
  g1s p = P[pair], o;
  if (!NORM) {  // the (x, y, c) form as it is
    o = p;
  } else if (fp_is_zero(p.c)) {
    fp_zero(o.x);
    fp_zero(o.y);
    fp_zero(o.c);
  } else {
    constexpr fp K8 = {{0x0347fcb8u, 0x19d80000u, 0x6d2002b1u, 0x12e00cdeu, 0xa2090c72u, 0x37669f83u,
                        0xda0f73e0u, 0x09b09b42u, 0x8f1297bbu, 0xa7c515d9u, 0xfcfa012cu, 0x0577a659u}};  // 2^8 R
    fp inv;
    fp_inv(inv, p.c);
    fp_mul(inv, inv, K8);  // 2^8 / c
    fp_mul(o.x, p.x, inv);
    fp_mul(o.y, p.y, inv);
    fp_one(o.c);
  }
  const uint32_t *w = reinterpret_cast<const uint32_t *>(&o);
#pragma unroll
  for (int i = 0; i < 36; i++) Pc[(size_t)i * ncol + c] = w[i];
}
void launch_ml_pcols(hipStream_t st, const g1s *P, const uint32_t *col, uint32_t np, uint32_t ncol,
                     uint32_t *Pc, bool normalize) {
  if (!np) return;
  if (normalize)
    k_ml_pcols<true><<<nblk(np), WG, 0, st>>>(P, col, np, ncol, Pc);
  else
    k_ml_pcols<false><<<nblk(np), WG, 0, st>>>(P, col, np, ncol, Pc);
}
void launch_ml_group(hipStream_t st, const uint32_t *lines, LineCols lc, uint32_t ngp, const g1s *P,
                     const uint32_t *Pc, const uint32_t *plist, const uint32_t *groups, uint32_t ngroup, int e0,
                     int e1, fp12 *V0, uint32_t *V28, bool pcn) {
  dim3 grid(nblk(ngroup), e1 - e0);
  if (!ngroup || e1 <= e0) return;
  const dim3 grid1(nblk(ngroup) * (uint32_t)(e1 - e0));
  if (g_ml_r28 && V28) {
    if (g_ml_dma)
      k_ml_group28<true, false><<<grid1, WG, 0, st>>>(lines, lc, ngp, P, Pc, plist, groups, ngroup, e0, e1 - e0, (int)g_ml_xcd, V28);
    else if (g_ml_kara && pcn)
      k_ml_group28<false, false, true, true><<<grid1, WG, 0, st>>>(lines, lc, ngp, P, Pc, plist, groups, ngroup, e0, e1 - e0, (int)g_ml_xcd, V28);
    else if (g_ml_kara)
      k_ml_group28<false, false, true><<<grid1, WG, 0, st>>>(lines, lc, ngp, P, Pc, plist, groups, ngroup, e0, e1 - e0, (int)g_ml_xcd, V28);
    else if (g_ml_prefetch && pcn)  // the points by column, normalized (k_ml_pcols): 4-product lines
      k_ml_group28<false, true, false, true><<<grid1, WG, 0, st>>>(lines, lc, ngp, P, Pc, plist, groups, ngroup, e0, e1 - e0, (int)g_ml_xcd, V28);
    else if (g_ml_prefetch)
      k_ml_group28<false, true><<<grid1, WG, 0, st>>>(lines, lc, ngp, P, Pc, plist, groups, ngroup, e0, e1 - e0, (int)g_ml_xcd, V28);
    else if (pcn)
      k_ml_group28<false, false, false, true><<<grid1, WG, 0, st>>>(lines, lc, ngp, P, Pc, plist, groups, ngroup, e0, e1 - e0, (int)g_ml_xcd, V28);
    else
      k_ml_group28<false, false><<<grid1, WG, 0, st>>>(lines, lc, ngp, P, Pc, plist, groups, ngroup, e0, e1 - e0, (int)g_ml_xcd, V28);
    const uint32_t nvals = ngroup * (uint32_t)(e1 - e0);
    k_ml_pack28<<<nblk((size_t)nvals * 12), WG, 0, st>>>(V28, ngroup, e0, nvals, V0);
    return;
  }
  k_ml_group<<<grid1, WG, 0, st>>>(lines, lc, ngp, P, plist, groups, ngroup, e0, e1 - e0, (int)g_ml_xcd, V0);
}
void launch_ml_reduce(hipStream_t st, const fp12 *Vin, uint32_t nin, const uint32_t *red,
                      uint32_t nout, fp12 *Vout) {
  dim3 grid(nout, ML_EVENTS);
  if (nout) k_ml_reduce<<<grid, 64, 0, st>>>(Vin, nin, red, nout, Vout);
}
// k_ml_horner on the row-distributed Fp12 engine (bls_w12d.h), for launches of a few
// segments, with the 68-event chain SPLIT into parts that run side by side (one workgroup
// each, grid (nseg, parts)): f = prod_k V_k^(2^(D_k)) (D_k = doubling events after k), so part
// [a, b) computes its own Horner value and then squares it once per doubling event after b;
// the parts' products are f.  With 4 parts the longest chain is 53.5 product-times instead of
// 113.5 (squarings at 0.75; tools/gpu notes in DESIGN.md section 9), and k_ml_combine_d
// multiplies the 4 values.  Event values are read as repacked limbs (an Fp* scalar each; the
// final exponentiation removes them); every part is conj'd (conj is a field automorphism).
struct HornerParts {
  int n;
  int b[8];  // part p covers events [b[p], b[p + 1])
};
constexpr HornerParts kHornerParts4 = {4, {0, 7, 18, 36, 68, 68, 68, 68}};
constexpr HornerParts kHornerParts1 = {1, {0, 68, 68, 68, 68, 68, 68, 68}};

__global__ void __launch_bounds__(w12d::THREADS) k_ml_horner_d(const fp12 *V, uint32_t nseg,
                                                               fp12 *out, const uint32_t *lim,
                                                               uint32_t base, HornerParts hp) {
  __shared__ __attribute__((aligned(16))) uint32_t ev[ML_EVENTS * w12d::IMG], acc[w12d::IMG],
      ws[w12d::WS];
  const uint32_t s = blockIdx.x, part = blockIdx.y;
  if (lim && base + s >= *lim) return;  // block-uniform
  const int e0 = hp.b[part], e1 = hp.b[part + 1];
  w12d::Eng e;
  w12d::begin(e, ws);
  for (uint32_t q = e.row; q < (uint32_t)(e1 - e0) * 12; q += w12d::ROWS) {
    const uint32_t ev_i = q / 12, c = q % 12;
    const uint32_t *w = reinterpret_cast<const uint32_t *>(V + (size_t)(e0 + ev_i) * nseg + s) + 12 * c;
    ev[ev_i * w12d::IMG + 16 * c + e.j] = dfp::from_words_scaled(w);
  }
  __syncthreads();
  w12d::copy(e, acc, ev);
  for (int k = e0 + 1; k < e1; k++) {
    if (ev_is_dbl(k)) w12d::sqr(e, acc, acc);
    w12d::mul(e, acc, acc, ev + (k - e0) * w12d::IMG);
  }
  for (int k = e1; k < ML_EVENTS; k++)
    if (ev_is_dbl(k)) w12d::sqr(e, acc, acc);
  w12d::conj(e, acc, acc);
  w12d::store_words(e, reinterpret_cast<uint32_t *>(out + (size_t)part * nseg + s), acc);
}
// partial[s] = prod_p parts[p][s] (row engine; canonical words out)
__global__ void __launch_bounds__(w12d::THREADS) k_ml_combine_d(const fp12 *parts, uint32_t nparts,
                                                                uint32_t nseg, fp12 *partial,
                                                                const uint32_t *lim, uint32_t base) {
  __shared__ __attribute__((aligned(16))) uint32_t acc[w12d::IMG], tmp[w12d::IMG], ws[w12d::WS];
  const uint32_t s = blockIdx.x;
  if (lim && base + s >= *lim) return;  // block-uniform
  w12d::Eng e;
  w12d::begin(e, ws);
  w12d::load_scaled(e, acc, reinterpret_cast<const uint32_t *>(parts + s));
  for (uint32_t p = 1; p < nparts; p++) {
    w12d::load_scaled(e, tmp, reinterpret_cast<const uint32_t *>(parts + (size_t)p * nseg + s));
    w12d::mul(e, acc, acc, tmp);
  }
  w12d::store_words(e, reinterpret_cast<uint32_t *>(partial + s), acc);
}

// segments up to this many take the row-distributed (latency) form
constexpr uint32_t kHornerRowsMaxSegs = 64;

void launch_ml_horner(hipStream_t st, const fp12 *V, uint32_t nseg, fp12 *partial,
                      const uint32_t *lim, uint32_t base, fp12 *tmp) {
  if (!nseg) return;
  if (nseg <= kHornerRowsMaxSegs && tmp) {
    k_ml_horner_d<<<dim3(nseg, kHornerParts4.n), w12d::THREADS, 0, st>>>(V, nseg, tmp, lim, base, kHornerParts4);
    k_ml_combine_d<<<nseg, w12d::THREADS, 0, st>>>(tmp, kHornerParts4.n, nseg, partial, lim, base);
  } else if (nseg <= kHornerRowsMaxSegs) {
    k_ml_horner_d<<<dim3(nseg, 1), w12d::THREADS, 0, st>>>(V, nseg, partial, lim, base, kHornerParts1);
  } else {
    k_ml_horner<<<nseg, 64, 0, st>>>(V, nseg, partial, lim, base);
  }
}

}  // namespace gbls
