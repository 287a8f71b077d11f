// gfx950 kernels: the random linear combination S = sum_i r_i sig_i of
// Signature::multi_verify (bls/src/signature.rs:117-126; blst accumulates it with one
// 64-bit POINTonE2_mult_w5 per set) as a bucket (Pippenger) multi-scalar multiplication,
// per segment of batches whose segments hold >= kMsmMinPerSeg sets (the C5-scale shards,
// coalesced C2 batches), where it replaces the per-set double-and-add of k_mv_g2mul and
// the chunk sums of k_g2sum: about W additions per set instead of 64 doublings + 32
// additions.  Point operations run on DPP quads (bls_gang.h) when the launch is small
// (latency regime) and one per lane when it fills the chip.
//
// Signed c-bit digits, W = ceil(65 / c) windows, B = 2^(c-1) buckets per window and
// segment (digit d != 0 adds sign(d) sig into bucket |d| - 1 of its segment's window):
//   1 k_msm_count    lane per set: bucket histogram (atomics)
//   2 k_msm_scan     one workgroup: bucket starts, chunk starts (K entries per chunk)
//   3 k_msm_scatter  lane per set: (set | sign) into its buckets' lists
//   4 k_msm_chunk    per chunk: sum of <= K affine points
//   5 k_msm_fold     per-bucket pairwise reduction of the chunk sums (log passes);
//     k_msm_bucket   the bucket sums as level-0 tree nodes
//   6 k_msm_tree     per (segment, window), a binary tree over the buckets computing
//                    S_w = sum_b (b+1) X_b with nodes (T = sum X, A = sum (b - lo) X):
//                    T = T_L + T_R, A = A_L + A_R + 2^l T_R   (l = level)
//   7 k_msm_final    quad per segment: S = sum_w 2^(c w) S_w (Horner), affine, the
//                    segment's extra pair (-g1, S)
// Infinite signatures and zero scalars contribute nothing (blst skips infinite
// signatures; a zero scalar fails the batch through k_msm_flags).  Bucket order is
// nondeterministic (atomics) but the sum is exact, so S is bit-exact.
#include "gbls_common.h"
#include "bls_gang.h"

namespace gbls {

constexpr int MSM_K = 16;  // points per chunk

__device__ __forceinline__ int msm_digit(uint64_t k, int w, int c, uint32_t &carry) {
  uint64_t raw = (c * w < 64) ? (k >> (c * w)) & ((1ull << c) - 1) : 0;
  int d = (int)raw + (int)carry;
  if (d > (1 << (c - 1))) {
    d -= 1 << c;
    carry = 1;
  } else {
    carry = 0;
  }
  return d;
}
// segment of set i: the largest s with seg_off[s] <= i (seg_off has nseg + 1 entries)
__device__ __forceinline__ uint32_t msm_segment(const uint32_t *seg_off, uint32_t nseg, uint32_t i) {
  uint32_t lo = 0, hi = nseg;
  while (hi - lo > 1) {
    uint32_t mid = (lo + hi) >> 1;
    if (seg_off[mid] <= i)
      lo = mid;
    else
      hi = mid;
  }
  return lo;
}

__global__ void __launch_bounds__(WGR) k_msm_count(const g2a *sigs, const uint64_t *rands, uint32_t n,
                                                   const uint32_t *seg_off, uint32_t nseg, int c,
                                                   int W, uint32_t *cnt) {
  uint32_t i = blockIdx.x * WGR + threadIdx.x;
  if (i >= n) return;
  uint64_t k = rands[i];
  if (k == 0 || aff_is_inf(sigs[i])) return;
  const uint32_t B = 1u << (c - 1);
  const uint32_t base = msm_segment(seg_off, nseg, i) * (uint32_t)W * B;
  uint32_t carry = 0;
  for (int w = 0; w < W; w++) {
    int d = msm_digit(k, w, c, carry);
    if (d) atomicAdd(&cnt[base + w * B + (uint32_t)(d < 0 ? -d : d) - 1], 1u);
  }
}

// one workgroup of 1024 lanes: start[b] (exclusive scan of cnt), cur = start,
// cstart[b] (exclusive scan of ceil(cnt / K)); start/cstart have nb + 1 entries
__global__ void __launch_bounds__(1024) k_msm_scan(const uint32_t *cnt, uint32_t nb, uint32_t *start,
                                                   uint32_t *cur, uint32_t *cstart) {
  __shared__ uint32_t s_a[1024], s_b[1024];
  __shared__ uint32_t base_a, base_b;
  if (threadIdx.x == 0) {
    base_a = 0;
    base_b = 0;
  }
  __syncthreads();
  for (uint32_t off = 0; off < nb; off += 1024) {
    uint32_t b = off + threadIdx.x;
    uint32_t x = b < nb ? cnt[b] : 0, y = (x + MSM_K - 1) / MSM_K;
    s_a[threadIdx.x] = x;
    s_b[threadIdx.x] = y;
    __syncthreads();
    for (uint32_t d = 1; d < 1024; d <<= 1) {  // inclusive Hillis-Steele scan
      uint32_t xa = threadIdx.x >= d ? s_a[threadIdx.x - d] : 0;
      uint32_t xb = threadIdx.x >= d ? s_b[threadIdx.x - d] : 0;
      __syncthreads();
      s_a[threadIdx.x] += xa;
      s_b[threadIdx.x] += xb;
      __syncthreads();
    }
    if (b < nb) {
      uint32_t sa = base_a + s_a[threadIdx.x] - x, sb = base_b + s_b[threadIdx.x] - y;
      start[b] = sa;
      cur[b] = sa;
      cstart[b] = sb;
    }
    __syncthreads();
    if (threadIdx.x == 1023) {
      base_a += s_a[1023];
      base_b += s_b[1023];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    start[nb] = base_a;
    cstart[nb] = base_b;
  }
}

__global__ void __launch_bounds__(WGR) k_msm_scatter(const g2a *sigs, const uint64_t *rands,
                                                     uint32_t n, const uint32_t *seg_off,
                                                     uint32_t nseg, int c, int W, uint32_t *cur,
                                                     uint32_t *list) {
  uint32_t i = blockIdx.x * WGR + threadIdx.x;
  if (i >= n) return;
  uint64_t k = rands[i];
  if (k == 0 || aff_is_inf(sigs[i])) return;
  const uint32_t B = 1u << (c - 1);
  const uint32_t base = msm_segment(seg_off, nseg, i) * (uint32_t)W * B;
  uint32_t carry = 0;
  for (int w = 0; w < W; w++) {
    int d = msm_digit(k, w, c, carry);
    if (!d) continue;
    uint32_t pos = atomicAdd(&cur[base + w * B + (uint32_t)(d < 0 ? -d : d) - 1], 1u);
    list[pos] = i | (d < 0 ? 0x80000000u : 0u);
  }
}

// point operations of the MSM kernels: on a DPP quad (Q, latency regime) or one lane
template <bool Q>
__device__ __forceinline__ void p_add(g2j &r, const g2j &a, const g2j &b, int q) {
  if (Q) {
    gang_add(r, a, b, q);
  } else {
    g2j t = b;
    jac_add(r, a, t);
  }
}
template <bool Q>
__device__ __forceinline__ void p_dbl(g2j &r, const g2j &a, int q) {
  if (Q)
    gang_dbl(r, a, q);
  else
    jac_dbl(r, a);
}
template <bool Q>
__device__ __forceinline__ uint32_t p_unit(int &q) {
  uint32_t t = blockIdx.x * WG + threadIdx.x;
  q = Q ? (int)(t & 3) : 0;
  return Q ? t >> 2 : t;
}

// chunk j: sum of <= K affine points of one bucket (found by binary search over cstart)
template <bool Q>
__global__ void __launch_bounds__(WG) k_msm_chunk(const g2a *sigs, const uint32_t *list,
                                                  const uint32_t *start, const uint32_t *cstart,
                                                  uint32_t nb, uint32_t max_chunks, g2j *chunk) {
  int q;
  uint32_t j = p_unit<Q>(q);
  if (j >= max_chunks || j >= cstart[nb]) return;  // whole quads
  uint32_t lo = 0, hi = nb;  // largest b with cstart[b] <= j
  while (hi - lo > 1) {
    uint32_t mid = (lo + hi) >> 1;
    if (cstart[mid] <= j)
      lo = mid;
    else
      hi = mid;
  }
  uint32_t b = lo;
  uint32_t e0 = start[b] + (j - cstart[b]) * MSM_K;
  uint32_t e1 = min(e0 + MSM_K, start[b + 1]);
  g2j acc;
  jac_set_inf(acc);
  for (uint32_t e = e0; e < e1; e++) {
    uint32_t v = list[e];
    g2a p = sigs[v & 0x7fffffffu];
    if (v >> 31) fp2_neg(p.y, p.y);
    if (Q) {
      g2j pj;
      jac_from_aff(pj, p);
      gang_add(acc, acc, pj, q);
    } else {
      jac_add_aff(acc, acc, p);
    }
  }
  if (q == 0) chunk[j] = acc;
}

// pass p of the per-bucket pairwise reduction of chunk sums: chunk k of bucket b (k a
// multiple of 2^(p+1)) absorbs chunk k + 2^p; log2(max chunks per bucket) passes leave
// every bucket's sum in its first chunk (depth log, whatever the digit distribution)
template <bool Q>
__global__ void __launch_bounds__(WG) k_msm_fold(const uint32_t *cstart, uint32_t nb,
                                                 uint32_t max_chunks, int p, g2j *chunk) {
  int q;
  uint32_t j = p_unit<Q>(q);
  if (j >= max_chunks || j >= cstart[nb]) return;
  uint32_t lo = 0, hi = nb;
  while (hi - lo > 1) {
    uint32_t mid = (lo + hi) >> 1;
    if (cstart[mid] <= j)
      lo = mid;
    else
      hi = mid;
  }
  uint32_t k = j - cstart[lo], step = 1u << p;
  if ((k & (2 * step - 1)) != 0 || j + step >= cstart[lo + 1]) return;
  g2j a = chunk[j], x = chunk[j + step];
  p_add<Q>(a, a, x, q);
  if (q == 0) chunk[j] = a;
}

// level-0 tree nodes: T = X_b (the bucket's folded first chunk, or infinity), A = inf
__global__ void __launch_bounds__(WG) k_msm_bucket(const g2j *chunk, const uint32_t *cstart,
                                                   uint32_t nb, g2j *T, g2j *A) {
  uint32_t b = blockIdx.x * WG + threadIdx.x;
  if (b >= nb) return;
  g2j inf;
  jac_set_inf(inf);
  T[b] = cstart[b + 1] > cstart[b] ? chunk[cstart[b]] : inf;
  A[b] = inf;
}

// tree level l: nodes (T, A) of ranges of 2^l buckets -> ranges of 2^(l+1); per
// (segment, window) group g the level has m = B >> (l+1) output nodes: inputs at
// g * 2m + 2q (+1), output at g * m + q.
template <bool Q>
__global__ void __launch_bounds__(WG) k_msm_tree(const g2j *Tin, const g2j *Ain, uint32_t groups,
                                                 uint32_t m, int l, g2j *Tout, g2j *Aout) {
  int q;
  uint32_t t = p_unit<Q>(q);
  if (t >= groups * m) return;
  uint32_t g = t / m, k2 = t % m;
  size_t li = (size_t)g * 2 * m + 2 * k2;
  g2j TL = Tin[li], TR = Tin[li + 1], AL = Ain[li], AR = Ain[li + 1];
  p_add<Q>(AL, AL, AR, q);
  g2j x = TR;
  for (int i = 0; i < l; i++) p_dbl<Q>(x, x, q);
  p_add<Q>(AL, AL, x, q);
  p_add<Q>(TL, TL, TR, q);
  if (q != 0) return;
  Tout[t] = TL;
  Aout[t] = AL;
}

// quad per segment: S_w = A_w + T_w (weights b + 1), S = sum_w 2^(c w) S_w, affine; the
// segment's extra Miller pair (-g1, S) at index n + s; an empty segment is flagged when
// empty_is_error
__global__ void __launch_bounds__(WG) k_msm_final(const g2j *T, const g2j *A, uint32_t nseg, int W,
                                                  int c, uint32_t n, const uint32_t *seg_off,
                                                  int empty_is_error, g1s *P, g2a *H,
                                                  int32_t *seg_err) {
  uint32_t s = (blockIdx.x * WG + threadIdx.x) >> 2;
  int q = (int)(threadIdx.x & 3);
  if (s >= nseg) return;
  g2j acc;
  jac_set_inf(acc);
  for (int w = W - 1; w >= 0; w--) {
    for (int i = 0; i < c && w != W - 1; i++) gang_dbl(acc, acc, q);
    g2j a = A[(size_t)s * W + w], t = T[(size_t)s * W + w];
    gang_add(a, a, t, q);
    gang_add(acc, acc, a, q);
  }
  g2a a;
  jac_to_aff(a, acc);
  if (q != 0) return;
  g1s ng1;
  fp_set(ng1.x, k::G1X_M);
  fp_set(ng1.y, k::G1NEGY_M);
  fp_one(ng1.c);
  P[n + s] = ng1;
  H[n + s] = a;
  if (empty_is_error && seg_off[s + 1] == seg_off[s]) atomicOr(&seg_err[s], 1);
}

// per-segment error flags: an infinite key, a zero scalar or a failed pre-check
__global__ void __launch_bounds__(WGR) k_msm_flags(const g1a *pks, const uint64_t *rands,
                                                   const int32_t *pre, const int32_t *pre2,
                                                   uint32_t n, const uint32_t *seg_off,
                                                   uint32_t nseg, int32_t *seg_err) {
  uint32_t i = blockIdx.x * WGR + threadIdx.x;
  if (i >= n) return;
  if (aff_is_inf(pks[i]) || rands[i] == 0 || (pre && pre[i] != 0) || (pre2 && pre2[i] != 0))
    atomicOr(&seg_err[msm_segment(seg_off, nseg, i)], 1);
}

// ---------------------------------------------------------------- host side
// Window widths dividing 65 (64-bit scalars + the signed-digit carry), so that no window
// is nearly empty (a 2-bit top window would pile every set into two buckets): c = 5
// (13 windows, 16 buckets each) for segments up to 2^16 sets, else c = 13 (5 windows,
// 4096 buckets).  Quad gangs below kLaneRegimeSets sets in the launch, one lane per
// operation above.
MsmPlan msm_plan(uint32_t n, uint32_t nseg) {
  uint32_t avg = nseg ? n / nseg : n;
  MsmPlan p;
  p.nseg = nseg;
  p.c = avg >= (1u << 16) ? 13 : 5;
  p.W = 65 / p.c;
  p.quad = n < kLaneRegimeSets;
  p.nb = nseg * ((uint32_t)p.W << (p.c - 1));
  p.max_chunks = (uint32_t)(((uint64_t)p.W * n + MSM_K - 1) / MSM_K) + p.nb;
  p.folds = 0;
  while ((1u << p.folds) < (uint32_t)((avg + MSM_K - 1) / MSM_K)) p.folds++;
  size_t o = 0;
  auto take = [&](size_t bytes) {
    size_t at = o;
    o += (bytes + 255) & ~(size_t)255;
    return at;
  };
  p.o_cnt = take(p.nb * 4);
  p.o_start = take((p.nb + 1) * 4);
  p.o_cur = take(p.nb * 4);
  p.o_cstart = take((p.nb + 1) * 4);
  p.o_list = take((size_t)p.W * n * 4);
  p.o_chunk = take((size_t)p.max_chunks * sizeof(g2j));
  p.o_t0 = take((size_t)p.nb * sizeof(g2j));
  p.o_a0 = take((size_t)p.nb * sizeof(g2j));
  p.o_t1 = take((size_t)(p.nb / 2 + 1) * sizeof(g2j));
  p.o_a1 = take((size_t)(p.nb / 2 + 1) * sizeof(g2j));
  p.bytes = o;
  return p;
}

template <bool Q>
static void launch_msm_points(hipStream_t st, const MsmPlan &p, const g2a *sigs, uint32_t *list,
                              uint32_t *start, uint32_t *cstart, g2j *chunk, g2j **T, g2j **A,
                              int &src) {
  const size_t L = Q ? 4 : 1;
  k_msm_chunk<Q><<<nblk(L * p.max_chunks), WG, 0, st>>>(sigs, list, start, cstart, p.nb,
                                                        p.max_chunks, chunk);
  for (int f = 0; f < p.folds + 1; f++)  // + 1: the digit distribution is not exactly flat
    k_msm_fold<Q><<<nblk(L * p.max_chunks), WG, 0, st>>>(cstart, p.nb, p.max_chunks, f, chunk);
  k_msm_bucket<<<nblk(p.nb), WG, 0, st>>>(chunk, cstart, p.nb, T[0], A[0]);
  src = 0;
  const uint32_t B = 1u << (p.c - 1), groups = p.nseg * (uint32_t)p.W;
  for (int l = 0; (1u << (l + 1)) <= B; l++) {
    uint32_t m = B >> (l + 1);
    k_msm_tree<Q><<<nblk(L * groups * m), WG, 0, st>>>(T[src], A[src], groups, m, l, T[1 - src],
                                                       A[1 - src]);
    src = 1 - src;
  }
}

void launch_msm(hipStream_t st, const MsmPlan &p, uint8_t *ws, const g2a *sigs,
                const uint64_t *rands, uint32_t n, const uint32_t *seg_off, int empty_is_error,
                g2a *H, g1s *P, int32_t *seg_err) {
  uint32_t *cnt = reinterpret_cast<uint32_t *>(ws + p.o_cnt);
  uint32_t *start = reinterpret_cast<uint32_t *>(ws + p.o_start);
  uint32_t *cur = reinterpret_cast<uint32_t *>(ws + p.o_cur);
  uint32_t *cstart = reinterpret_cast<uint32_t *>(ws + p.o_cstart);
  uint32_t *list = reinterpret_cast<uint32_t *>(ws + p.o_list);
  g2j *chunk = reinterpret_cast<g2j *>(ws + p.o_chunk);
  g2j *T[2] = {reinterpret_cast<g2j *>(ws + p.o_t0), reinterpret_cast<g2j *>(ws + p.o_t1)};
  g2j *A[2] = {reinterpret_cast<g2j *>(ws + p.o_a0), reinterpret_cast<g2j *>(ws + p.o_a1)};
  (void)hipMemsetAsync(cnt, 0, p.nb * 4, st);
  (void)hipMemsetAsync(seg_err, 0, p.nseg * 4, st);
  k_msm_count<<<nblk(n, WGR), WGR, 0, st>>>(sigs, rands, n, seg_off, p.nseg, p.c, p.W, cnt);
  k_msm_scan<<<1, 1024, 0, st>>>(cnt, p.nb, start, cur, cstart);
  k_msm_scatter<<<nblk(n, WGR), WGR, 0, st>>>(sigs, rands, n, seg_off, p.nseg, p.c, p.W, cur,
                                              list);
  int src = 0;
  if (p.quad)
    launch_msm_points<true>(st, p, sigs, list, start, cstart, chunk, T, A, src);
  else
    launch_msm_points<false>(st, p, sigs, list, start, cstart, chunk, T, A, src);
  k_msm_final<<<nblk(4 * (size_t)p.nseg), WG, 0, st>>>(T[src], A[src], p.nseg, p.W, p.c, n,
                                                       seg_off, empty_is_error, P, H, seg_err);
}

void launch_msm_flags(hipStream_t st, const g1a *pks, const uint64_t *rands, const int32_t *pre,
                      const int32_t *pre2, uint32_t n, const uint32_t *seg_off, uint32_t nseg,
                      int32_t *seg_err) {
  if (n) k_msm_flags<<<nblk(n, WGR), WGR, 0, st>>>(pks, rands, pre, pre2, n, seg_off, nseg, seg_err);
}

}  // namespace gbls
