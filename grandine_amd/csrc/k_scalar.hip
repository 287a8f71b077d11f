// gfx950 kernels: the random linear combination of Signature::multi_verify
// (bls/src/signature.rs:106-126): P_i = r_i pk_i (G1, one lane per set) and
// S = sum r_i sig_i (G2).  The G2 side splits every 64-bit scalar into 32-bit halves
// (two lanes per set, half the serial chain): S = S_lo + [2^32] S_hi with
// S_lo = sum [lo(r_i)] sig_i, S_hi = sum [hi(r_i)] sig_i, summed by a two-level
// workgroup tree.
#include "gbls_common.h"
#include "bls_curve28.h"
#include "bls_gang.h"
#include "bls_w4.h"

namespace gbls {

// the wave-per-point (W4) kernels of this group live in k_scalar_w4.hip (a translation unit of
// their own, so the two compile in parallel)
void launch_mv_g1mul_w4(hipStream_t st, const g1a *pks, const uint64_t *rands, uint32_t n, g1s *P);
void launch_mv_g2mul_w4(hipStream_t st, const g2a *sigs, const uint64_t *rands, uint32_t n, g2j *R);
void launch_g2sum_final_w4(hipStream_t st, const g2j *part, const int32_t *part_err, const uint32_t *chunks,
                           const uint32_t *seg_chunk, const uint32_t *seg_off, uint32_t nseg, uint32_t n,
                           int empty_is_error, g1s *P, g2a *H, int32_t *seg_err, g2j *Sj);

// P_i = r_i pk_i as a line-evaluation point (x, y, c) = (X Z, Y, Z^3) of the Jacobian
// result (bls_pairing.h g1s): no inversion.  One DPP quad per set, MSB-first
// double-and-add with quad doublings / additions (bls_gang.h); lane 0 stores.
template <bool X>
__global__ void __launch_bounds__(WG) k_mv_g1mul(const g1a *pks, const uint64_t *rands, uint32_t n,
                                                 g1s *P) {
  if constexpr (X) w4::exclusive_simd();
  uint32_t u = blockIdx.x * WG + threadIdx.x;
  uint32_t i = u >> 2;
  int q = (int)(u & 3);
  if (i >= n) return;  // whole quads only
  g1a pk = pks[i];
  g1s o;
  if (!rands) {  // r = 1 (single checks): the key itself
    g1s_from_aff(o, pk);
    if (q == 0) P[i] = o;
    return;
  }
  uint64_t k = rands[i];
  g1j acc;
  jac_set_inf(acc);
  if (k != 0 && !aff_is_inf(pk)) {
    int top = 63;
    while (!((k >> top) & 1)) top--;
    g1j base;
    jac_from_aff(base, pk);
    acc = base;
    for (int b = top - 1; b >= 0; b--) {
      gang1_dbl(acc, acc, q);
      if ((k >> b) & 1) gang1_add(acc, acc, base, q);
    }
  }
  g1s_from_jac(o, acc);
  if (q == 0) P[i] = o;
}

// R[h * n + i] = [32-bit half h of r_i] sig_i (Jacobian); infinite signatures give the
// identity (blst skips them in the G2 accumulation)
// r.sigma, split into two 32-bit halves, each half on one DPP quad (quad doublings,
// bls_gang.h, and quad additions with Z2 = 1); lane 0 of the quad stores.
__global__ void __launch_bounds__(WG) k_mv_g2mul(const g2a *sigs, const uint64_t *rands, uint32_t n,
                                                 g2j *R) {
  uint32_t u = blockIdx.x * WG + threadIdx.x;
  uint32_t t = u >> 2;
  int q = (int)(u & 3);
  if (t >= 2 * n) return;  // whole quads only
  uint32_t i = t < n ? t : t - n;
  uint64_t r = rands ? rands[i] : 1;
  uint64_t k = t < n ? (r & 0xffffffffull) : (r >> 32);
  g2a base = sigs[i];
  g2j acc;
  jac_set_inf(acc);
  if (k != 0 && !aff_is_inf(base)) {
    int top = 63;
    while (!((k >> top) & 1)) top--;
    g2j bj;
    jac_from_aff(bj, base);
    acc = bj;
    for (int b = top - 1; b >= 0; b--) {
      gang_dbl(acc, acc, q);
      if ((k >> b) & 1) gang_add(acc, acc, bj, q);
    }
  }
  if (q == 0) R[t] = acc;
}


// level 1: workgroup c sums R[h*n + b .. h*n + e) (chunk table: {s, h, b, e}, at most
// WGR sets) with quad additions (bls_gang.h): each of the 64 quads folds a strided
// subset, then a 6-level LDS tree joins the quads.  It also ORs the bad flags: pk
// infinite (blst PAIRING_Aggregate_PK_in_G1), a zero scalar (the reference only draws
// NonZeroU64, signature.rs:106-115; a zero would drop the set from the combination, so
// it fails closed), or a failed pre-check
__global__ void __launch_bounds__(WGR) k_g2sum_chunks(const g2j *R, const uint32_t *chunks, uint32_t n,
                                                      const g1a *pks, const uint64_t *rands,
                                                      const int32_t *pre, const int32_t *pre2,
                                                      g2j *part, int32_t *part_err) {
  constexpr int NQ = WGR / 4;
  __shared__ g2j sh[NQ / 2];
  __shared__ int32_t e_sh;
  uint32_t c = blockIdx.x;
  uint32_t h = chunks[4 * c + 1], b = chunks[4 * c + 2], e = chunks[4 * c + 3];
  int w = (int)(threadIdx.x >> 2), q = (int)(threadIdx.x & 3);
  if (threadIdx.x == 0) e_sh = 0;
  __syncthreads();
  g2j acc;
  jac_set_inf(acc);
  int32_t bad = 0;
  for (uint32_t i = b + w; i < e; i += NQ) {
    g2j r = R[(size_t)h * n + i];
    gang_add(acc, acc, r, q);
    if (h == 0 && q == 0)
      bad |= ((pks && aff_is_inf(pks[i])) || (rands && rands[i] == 0) || (pre && pre[i] != 0) ||
              (pre2 && pre2[i] != 0))
                 ? 1
                 : 0;
  }
  if (bad) atomicOr(&e_sh, 1);
  for (int width = NQ / 2; width > 0; width >>= 1) {
    __syncthreads();
    if (q == 0 && w >= width && w < 2 * width) sh[w - width] = acc;
    __syncthreads();
    if (w < width) {
      g2j o = sh[w];
      gang_add(acc, acc, o, q);
    }
  }
  if (threadIdx.x == 0) {
    part[c] = acc;
    part_err[c] = e_sh;
  }
}

// the key-side flags of level 1's chunks (an infinite key, a failed key pre-check), ORed into
// part_err: lets level 1 start before the keys are resolved on the other side stream
__global__ void __launch_bounds__(WGR) k_g2sum_flags(const uint32_t *chunks, const g1a *pks,
                                                     const int32_t *pre, int32_t *part_err) {
  __shared__ int32_t e_sh;
  const uint32_t c = blockIdx.x;
  const uint32_t h = chunks[4 * c + 1], b = chunks[4 * c + 2], e = chunks[4 * c + 3];
  if (threadIdx.x == 0) e_sh = 0;
  __syncthreads();
  int32_t bad = 0;
  if (h == 0)
    for (uint32_t i = b + threadIdx.x; i < e; i += WGR)
      bad |= (aff_is_inf(pks[i]) || (pre && pre[i] != 0)) ? 1 : 0;
  if (bad) atomicOr(&e_sh, 1);
  __syncthreads();
  if (threadIdx.x == 0 && e_sh) part_err[c] |= 1;
}

// level 2: one lane per segment: S = S_lo + [2^32] S_hi over the segment's chunks, then
// the segment's extra Miller pair (-g1, S) at index n + s; seg_err[s] = OR bad | empty
// One wave per segment: 16 DPP quads each fold a strided subset of the segment's chunk
// partials (quad additions), then a 4-level LDS tree joins the 16 quads; quad 0 applies
// the 2^32 shift of the high halves and converts to affine.
__global__ void __launch_bounds__(WG) k_g2sum_final(const g2j *part, const int32_t *part_err,
                                                    const uint32_t *chunks, const uint32_t *seg_chunk,
                                                    const uint32_t *seg_off, uint32_t nseg, uint32_t n,
                                                    int empty_is_error, g1s *P, g2a *H,
                                                    int32_t *seg_err) {
  constexpr int NQ = WG / 4;
  __shared__ g2j sh_lo[NQ], sh_hi[NQ];
  __shared__ int32_t sh_err[NQ];
  uint32_t s = blockIdx.x;  // grid = nseg exactly
  int w = (int)(threadIdx.x >> 2), q = (int)(threadIdx.x & 3);
  g2j lo, hi;
  jac_set_inf(lo);
  jac_set_inf(hi);
  int32_t err = 0;
  for (uint32_t c = seg_chunk[s] + w; c < seg_chunk[s + 1]; c += NQ) {
    g2j v = part[c];
    if (chunks[4 * c + 1] == 0)
      gang_add(lo, lo, v, q);
    else
      gang_add(hi, hi, v, q);
    err |= part_err[c];
  }
  for (int width = NQ / 2; width > 0; width >>= 1) {
    __syncthreads();
    if (q == 0 && w >= width && w < 2 * width) {
      sh_lo[w - width] = lo;
      sh_hi[w - width] = hi;
      sh_err[w - width] = err;
    }
    __syncthreads();
    if (w < width) {
      g2j o = sh_lo[w];
      gang_add(lo, lo, o, q);
      o = sh_hi[w];
      gang_add(hi, hi, o, q);
      err |= sh_err[w];
    }
  }
  if (w != 0) return;
  if (empty_is_error && seg_off[s + 1] == seg_off[s]) err = 1;
  for (int j = 0; j < 32; j++) gang_dbl(hi, hi, q);
  gang_add(lo, lo, hi, q);
  g1s ng1;
  fp_set(ng1.x, k::G1X_M);
  fp_set(ng1.y, k::G1NEGY_M);
  fp_one(ng1.c);
  g2a a;
  jac_to_aff(a, lo);
  if (q != 0) return;
  P[n + s] = ng1;
  H[n + s] = a;
  seg_err[s] = err;
}

// Single checks (r_i = 1, one set per segment: verify / fast_aggregate_verify batches):
// S_s = sig_s, so the segment's extra pair is (-g1, sig_s) -- no G2 sum, no inversion.
__global__ void __launch_bounds__(WG) k_single_S(const g2a *sigs, const g1a *pks, const int32_t *pre,
                                                 const int32_t *pre2, uint32_t n, g1s *P, g2a *H,
                                                 int32_t *seg_err, g1a *ng1_out) {
  uint32_t s = blockIdx.x * WG + threadIdx.x;
  if (s >= n) return;
  if (ng1_out) {  // grouped checks: -g1 as the base of the scaled pair (k_mv_g1mul writes P)
    g1a a;
    fp_set(a.x, k::G1X_M);
    fp_set(a.y, k::G1NEGY_M);
    ng1_out[s] = a;
  } else {
    g1s ng1;
    fp_set(ng1.x, k::G1X_M);
    fp_set(ng1.y, k::G1NEGY_M);
    fp_one(ng1.c);
    P[n + s] = ng1;
  }
  H[n + s] = sigs[s];
  seg_err[s] = (aff_is_inf(pks[s]) || (pre && pre[s] != 0) || (pre2 && pre2[s] != 0)) ? 1 : 0;
}

void launch_single_S(hipStream_t st, const g2a *sigs, const g1a *pks, const int32_t *pre,
                     const int32_t *pre2, uint32_t n, g1s *P, g2a *H, int32_t *seg_err,
                     g1a *ng1_out) {
  if (n) k_single_S<<<nblk(n), WG, 0, st>>>(sigs, pks, pre, pre2, n, P, H, seg_err, ng1_out);
}

// grouped single checks: the error flag of each group of gs checks (any member's)
__global__ void __launch_bounds__(WG) k_group_err(const int32_t *err, uint32_t n, uint32_t gs,
                                                  uint32_t ngrp, int32_t *gerr) {
  const uint32_t gi = blockIdx.x * WG + threadIdx.x;
  if (gi >= ngrp) return;
  int32_t bad = 0;
  for (uint32_t i = gi * gs; i < min(n, (gi + 1) * gs); i++) bad |= err[i];
  gerr[gi] = bad;
}
void launch_group_err(hipStream_t st, const int32_t *err, uint32_t n, uint32_t gs, uint32_t ngrp,
                      int32_t *gerr) {
  if (ngrp) k_group_err<<<nblk(ngrp), WG, 0, st>>>(err, n, gs, ngrp, gerr);
}

// Throughput variant for large batches (every SIMD already busy): one lane per set,
// signed 3-bit windows (g1_mul_u64_w3: the same instructions for every lane's scalar).
__global__ void __launch_bounds__(WG) k_mv_g1mul_lane(const g1a *pks, const uint64_t *rands,
                                                      uint32_t n, g1s *P) {
  uint32_t i = blockIdx.x * WG + threadIdx.x;
  if (i >= n) return;
  g1a pk = pks[i];
  g1s o;
  if (!rands) {
    g1s_from_aff(o, pk);
  } else {
    g1j t;
    g1_mul_u64_w3(t, pk, rands[i]);
    g1s_from_jac(o, t);
  }
  P[i] = o;
}

// the same in radix 2^28 (bls_curve28.h g1_mul_u64_w3_28: one v_mad_u64_u32 per product term,
// squarings by the dedicated square), the default with the other radix-2^28 lanes (g_lane_r28)
__global__ void __launch_bounds__(WG) k_mv_g1mul_lane28(const g1a *pks, const uint64_t *rands,
                                                        uint32_t n, g1s *P) {
  uint32_t i = blockIdx.x * WG + threadIdx.x;
  if (i >= n) return;
  const g1a pk = pks[i];
  g1s o;
  if (!rands) {
    g1s_from_aff(o, pk);
  } else {
    r28::g1j28 t;
    r28::g1_mul_u64_w3_28(t, pk, rands[i]);
    r28::g1s_from_jac28(o, t);
  }
  P[i] = o;
}

void launch_mv_g1mul(hipStream_t st, const g1a *pks, const uint64_t *rands, uint32_t n, g1s *P) {
  if (!n) return;
  if (rands && n <= kW4Max) {
    launch_mv_g1mul_w4(st, pks, rands, n, P);
    return;
  }
  if (n >= g_lane_min && g_lane_r28)
    k_mv_g1mul_lane28<<<nblk(n), WG, 0, st>>>(pks, rands, n, P);
  else if (n >= g_lane_min)
    k_mv_g1mul_lane<<<nblk(n), WG, 0, st>>>(pks, rands, n, P);
  else
    (nblk(4 * (size_t)n) <= w4::kExclusiveMaxWaves ? k_mv_g1mul<true> : k_mv_g1mul<false>)<<<
        nblk(4 * (size_t)n), WG, 0, st>>>(pks, rands, n, P);
}
void launch_mv_g2mul(hipStream_t st, const g2a *sigs, const uint64_t *rands, uint32_t n, g2j *R) {
  if (!n) return;
  if (n <= kW4Max)  // 2n waves: up to two per SIMD, still ahead of the quads' one-lane chains
    launch_mv_g2mul_w4(st, sigs, rands, n, R);
  else
    k_mv_g2mul<<<nblk(8 * (size_t)n), WG, 0, st>>>(sigs, rands, n, R);
}
void launch_g2sum(hipStream_t st, const g2j *R, const uint32_t *chunks, uint32_t nchunks,
                  const uint32_t *seg_chunk, const uint32_t *seg_off, uint32_t nseg, uint32_t n,
                  const g1a *pks, const uint64_t *rands, const int32_t *pre, const int32_t *pre2,
                  int empty_is_error, g2j *part, int32_t *part_err, g1s *P, g2a *H,
                  int32_t *seg_err, g2j *Sj, hipEvent_t keys_ready) {
  if (keys_ready) {  // level 1 before the keys, their flags after
    if (nchunks) k_g2sum_chunks<<<nchunks, WGR, 0, st>>>(R, chunks, n, nullptr, rands, nullptr, pre2, part, part_err);
    (void)hipStreamWaitEvent(st, keys_ready, 0);
    if (nchunks) k_g2sum_flags<<<nchunks, WGR, 0, st>>>(chunks, pks, pre, part_err);
  } else if (nchunks) {
    k_g2sum_chunks<<<nchunks, WGR, 0, st>>>(R, chunks, n, pks, rands, pre, pre2, part, part_err);
  }

  if (nseg && nseg <= kW4Max)
    launch_g2sum_final_w4(st, part, part_err, chunks, seg_chunk, seg_off, nseg, n, empty_is_error, P, H, seg_err,
                          Sj);
  else if (nseg)
    k_g2sum_final<<<nseg, WG, 0, st>>>(part, part_err, chunks, seg_chunk, seg_off, nseg, n,
                                       empty_is_error, P, H, seg_err);
}

}  // namespace gbls
