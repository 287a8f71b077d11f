// gfx950 kernels: the random linear combination S = sum_i r_i sig_i of
// Signature::multi_verify (bls/src/signature.rs:117-126; blst accumulates it with one
// 64-bit POINTonE2_mult_w5 per set) as a bucket (Pippenger) multi-scalar multiplication,
// per segment of batches whose segments hold >= kMsmMinPerSeg sets (the C5-scale shards,
// coalesced C2 batches), where it replaces the per-set double-and-add of k_mv_g2mul and
// the chunk sums of k_g2sum: about W mixed additions per set instead of 64 doublings +
// 32 additions.
//
// Signed c-bit digits, W = 65 / c windows, B = 2^(c-1) buckets per window and segment
// (digit d != 0 adds sign(d) sig into bucket |d| - 1 of its segment's window):
//   1 k_msm_count    lane per set: bucket histogram (atomics), segment error flags
//   2 k_msm_scan     one workgroup: bucket starts, chunk starts (K entries per chunk)
//   3 k_msm_scatter  lane per set: (set | sign) into its buckets' lists
//   4 k_msm_chunk    lane per chunk: sum of <= K affine points (mixed additions), then a
//                    segmented fold of the wave's chunks by bucket through LDS (one
//                    partial per bucket and wave; the bucket's reader adds them up)
// The bucket sums X_{w,b} never go through a Horner chain of 60 doublings.  The weights
// move to the G1 side of the pairing instead, where they are constants:
//   e(-g1, S) = prod_{w,b} e(-[(b+1) 2^(c w)] g1, X_{w,b}),
// so every bucket becomes one extra Miller pair of its segment, with a precomputed G1
// point (bls_constants.h MSM_W5, tools/gen_constants.py).  With c = 5 that is
// 13 * 16 = 208 pairs per segment (+5% Miller work at 4096 sets), and the G2 side has
// no serial tail:
//   5 k_msm_pairs    lane per bucket: X_{w,b} (the bucket's partials), affine, its pair
// With c = 13 (segments >= 2^16 sets, 4096 buckets per window) a per-window tree
// first folds the weights (b + 1) into S_w, and the 5 window sums pair with
// -[2^(13 w)] g1 (MSM_W13):
//   5 k_msm_bucket   level-0 tree nodes (the buckets' partials added up)
//   6 k_msm_tree     per (segment, window), a binary tree over the buckets computing
//                    S_w = sum_b (b+1) X_b with nodes (T = sum X, A = sum (b - lo) X):
//                    T = T_L + T_R, A = A_L + A_R + 2^l T_R   (l = level)
//   7 k_msm_wpairs   lane per window: affine S_w = A + T, its pair
// Infinite signatures and zero scalars contribute nothing (blst skips infinite
// signatures; a zero scalar fails the batch through k_msm_count's flags).  An empty bucket is
// the point at infinity, whose Miller pair is the identity.  Bucket order is
// nondeterministic (atomics) but the sums are exact, so the verdict is too.
#include "gbls_common.h"
#include "bls_gang.h"

namespace gbls {


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

// also the per-segment error flags: an infinite key, a zero scalar or a failed
// pre-check (key aggregation / signature group check) fails the set's segment
__global__ void __launch_bounds__(WGR) k_msm_count(const g2a *sigs, const uint64_t *rands, uint32_t n,
                                                   const uint32_t *seg_off, uint32_t nseg, int c,
                                                   int W, const g1a *pks, const int32_t *pre,
                                                   const int32_t *pre2, uint32_t *cnt,
                                                   int32_t *seg_err) {
  uint32_t i = blockIdx.x * WGR + threadIdx.x;
  if (i >= n) return;
  uint64_t k = rands[i];
  const uint32_t s = msm_segment(seg_off, nseg, i);
  if (aff_is_inf(pks[i]) || k == 0 || (pre && pre[i] != 0) || (pre2 && pre2[i] != 0))
    atomicOr(&seg_err[s], 1);
  if (k == 0 || aff_is_inf(sigs[i])) return;
  const uint32_t B = 1u << (c - 1);
  const uint32_t base = s * (uint32_t)W * B;
  uint32_t carry = 0;
  for (int w = 0; w < W; w++) {
    int d = msm_digit(k, w, c, carry);
    if (d) atomicAdd(&cnt[base + w * B + (uint32_t)(d < 0 ? -d : d) - 1], 1u);
  }
}

// one workgroup of 1024 lanes: start[b] (exclusive scan of cnt), cur = start,
// cstart[b] (exclusive scan of ceil(cnt / K)); start/cstart have nb + 1 entries
__global__ void __launch_bounds__(1024) k_msm_scan(const uint32_t *cnt, uint32_t nb, uint32_t K,
                                                   uint32_t *start, uint32_t *cur, uint32_t *cstart) {
  __shared__ uint32_t s_a[1024], s_b[1024];
  __shared__ uint32_t base_a, base_b;
  if (threadIdx.x == 0) {
    base_a = 0;
    base_b = 0;
  }
  __syncthreads();
  for (uint32_t off = 0; off < nb; off += 1024) {
    uint32_t b = off + threadIdx.x;
    uint32_t x = b < nb ? cnt[b] : 0, y = (x + K - 1) / K;
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

// chunk j: sum of <= K affine points of one bucket (found by binary search over cstart),
// then, within the wave, a segmented pairwise fold of the wave's chunks by bucket: every
// bucket's chunks inside one wave end up summed in its first chunk there (levels only
// while some run of same-bucket chunks in the wave is longer than the step).  A bucket
// thus leaves one partial per wave it touches, at its first chunk cstart[b] and at each
// wave boundary 64 w inside [cstart[b], cstart[b + 1]) (msm_bucket_sum).
__global__ void __launch_bounds__(WG) k_msm_chunk(const g2a *sigs, const uint32_t *list,
                                                  const uint32_t *start, const uint32_t *cstart,
                                                  uint32_t nb, uint32_t max_chunks, uint32_t K,
                                                  g2j *chunk) {
  // structure-of-arrays image of the wave's partials: word w of lane l at xs[w * WG + l], so a
  // wave's 64 lanes touch 64 consecutive words (distinct banks) on every store and load (the
  // array-of-structures image, 288-byte stride, put 16 lanes on each bank: 80 % of the LDS
  // cycles were conflicts)
  constexpr int NW = sizeof(g2j) / 4;
  __shared__ uint32_t xs[NW * WG];
  const uint32_t lane = threadIdx.x, base = blockIdx.x * WG;
  const uint32_t j = base + lane, total = cstart[nb];
  const bool live = j < max_chunks && j < total;
  g2j acc;
  jac_set_inf(acc);
  uint32_t lo = 0;
  if (live) {
    uint32_t hi = nb;  // largest b with cstart[b] <= j
    while (hi - lo > 1) {
      uint32_t mid = (lo + hi) >> 1;
      if (cstart[mid] <= j)
        lo = mid;
      else
        hi = mid;
    }
    uint32_t e0 = start[lo] + (j - cstart[lo]) * K;
    uint32_t e1 = min(e0 + K, start[lo + 1]);
    // the next point's loads are issued before this point's addition: at one wave per SIMD the
    // chain otherwise waits on every random-address load (VALU busy 0.43 in the r04 PMC pass)
    uint32_t vn = list[e0];
    g2a pn = sigs[vn & 0x7fffffffu];
    for (uint32_t e = e0; e < e1; e++) {
      const uint32_t v = vn;
      g2a p = pn;
      if (e + 1 < e1) {
        vn = list[e + 1];
        pn = sigs[vn & 0x7fffffffu];
      }
      if (v >> 31) fp2_neg(p.y, p.y);
      jac_add_aff(acc, acc, p);
    }
  }
  // this lane's position in its bucket's run inside the wave, and the run's end (lanes)
  const uint32_t first = live ? (cstart[lo] > base ? cstart[lo] - base : 0u) : lane;
  const uint32_t end = live ? min((uint32_t)WG, cstart[lo + 1] - base) : lane + 1;
  const uint32_t k = lane - first;
  uint32_t run = end - first;  // wave maximum of the run lengths
  for (int o = 32; o >= 1; o >>= 1) run = max(run, (uint32_t)__shfl_xor((int)run, o));
  for (uint32_t st = 1; st < run; st <<= 1) {
    const uint32_t *aw = reinterpret_cast<const uint32_t *>(&acc);
#pragma unroll
    for (int w = 0; w < NW; w++) xs[w * WG + lane] = aw[w];
    __syncthreads();
    if ((k & (2 * st - 1)) == 0 && lane + st < end) {
      g2j x;
      uint32_t *xw = reinterpret_cast<uint32_t *>(&x);
#pragma unroll
      for (int w = 0; w < NW; w++) xw[w] = xs[w * WG + lane + st];
      jac_add(acc, acc, x);
    }
    __syncthreads();
  }
  if (live && k == 0) chunk[j] = acc;
}

// sum of bucket b: its first chunk's partial plus the partials at the chunk waves' starts
// inside the bucket's chunk range (k_msm_chunk)
__device__ __forceinline__ void msm_bucket_sum(g2j &x, const g2j *chunk, const uint32_t *cstart,
                                               uint32_t b) {
  const uint32_t c0 = cstart[b], c1 = cstart[b + 1];
  if (c1 == c0) {
    jac_set_inf(x);
    return;
  }
  x = chunk[c0];
  for (uint32_t w = (c0 / WG + 1) * WG; w < c1; w += WG) {
    g2j y = chunk[w];
    jac_add(x, x, y);
  }
}

// the constant G1 half of an extra pair: table entry k (x, y Montgomery), c = 1
__device__ __forceinline__ void msm_weight(g1s &o, const uint32_t *table, uint32_t k) {
#pragma unroll
  for (int i = 0; i < 12; i++) {
    o.x.l[i] = table[24 * k + i];
    o.y.l[i] = table[24 * k + 12 + i];
  }
  fp_one(o.c);
}

// c = 5: lane per bucket t = s * W * B + k; its sum X (the bucket's folded first chunk, or
// infinity) pairs with -[(b+1) 2^(c w)] g1 at pair n + t
__global__ void __launch_bounds__(WG) k_msm_pairs(const g2j *chunk, const uint32_t *cstart,
                                                  uint32_t nb, uint32_t per_seg, uint32_t n,
                                                  const uint32_t *seg_off, int empty_is_error,
                                                  g1s *P, g2a *H, int32_t *seg_err) {
  uint32_t t = blockIdx.x * WG + threadIdx.x;
  if (t >= nb) return;
  uint32_t s = t / per_seg, k = t % per_seg;
  g2j x;
  msm_bucket_sum(x, chunk, cstart, t);
  g2a a;
  jac_to_aff(a, x);
  g1s w;
  msm_weight(w, k::MSM_W5, k);
  P[n + t] = w;
  H[n + t] = a;
  if (k == 0 && empty_is_error && seg_off[s + 1] == seg_off[s]) atomicOr(&seg_err[s], 1);
}

// level-0 tree nodes: T = X_b (the bucket's folded first chunk, or infinity), A = inf
__global__ void __launch_bounds__(WG) k_msm_bucket(const g2j *chunk, const uint32_t *cstart,
                                                   uint32_t nb, g2j *T, g2j *A) {
  uint32_t b = blockIdx.x * WG + threadIdx.x;
  if (b >= nb) return;
  g2j x, inf;
  msm_bucket_sum(x, chunk, cstart, b);
  jac_set_inf(inf);
  T[b] = x;
  A[b] = inf;
}

// tree level l: nodes (T, A) of ranges of 2^l buckets -> ranges of 2^(l+1); per
// (segment, window) group g the level has m = B >> (l+1) output nodes: inputs at
// g * 2m + 2q (+1), output at g * m + q.
__global__ void __launch_bounds__(WG) k_msm_tree(const g2j *Tin, const g2j *Ain, uint32_t groups,
                                                 uint32_t m, int l, g2j *Tout, g2j *Aout) {
  uint32_t t = blockIdx.x * WG + threadIdx.x;
  if (t >= groups * m) return;
  uint32_t g = t / m, k2 = t % m;
  size_t li = (size_t)g * 2 * m + 2 * k2;
  g2j TL = Tin[li], TR = Tin[li + 1], AL = Ain[li], AR = Ain[li + 1];
  jac_add(AL, AL, AR);
  g2j x = TR;
  for (int i = 0; i < l; i++) jac_dbl(x, x);
  jac_add(AL, AL, x);
  jac_add(TL, TL, TR);
  Tout[t] = TL;
  Aout[t] = AL;
}

// c = 13: lane per (segment, window) t = s * W + w: S_w = A_w + T_w (weights b + 1),
// affine, paired with -[2^(c w)] g1 at pair n + t
__global__ void __launch_bounds__(WG) k_msm_wpairs(const g2j *T, const g2j *A, uint32_t nw,
                                                   uint32_t W, uint32_t n, const uint32_t *seg_off,
                                                   int empty_is_error, g1s *P, g2a *H,
                                                   int32_t *seg_err) {
  uint32_t t = blockIdx.x * WG + threadIdx.x;
  if (t >= nw) return;
  uint32_t s = t / W, w = t % W;
  g2j a = A[t], b = T[t];
  jac_add(a, a, b);
  g2a o;
  jac_to_aff(o, a);
  g1s g;
  msm_weight(g, k::MSM_W13, w);
  P[n + t] = g;
  H[n + t] = o;
  if (w == 0 && empty_is_error && seg_off[s + 1] == seg_off[s]) atomicOr(&seg_err[s], 1);
}

// ---------------------------------------------------------------- host side
// Window widths dividing 65 (64-bit scalars + the signed-digit carry), so that no window
// is nearly empty (a 2-bit top window would pile every set into two buckets): c = 5
// (13 windows, 16 buckets each, one Miller pair per bucket) for segments up to 2^16 sets,
// else c = 13 (5 windows of 4096 buckets, per-window trees, one pair per window).
MsmPlan msm_plan(uint32_t n, uint32_t nseg) {
  uint32_t avg = nseg ? n / nseg : n;
  MsmPlan p;
  p.nseg = nseg;
  p.c = avg >= (1u << 16) ? 13 : 5;
  p.W = 65 / p.c;
  p.tree = p.c == 13;
  p.extra = p.tree ? (uint32_t)p.W : ((uint32_t)p.W << (p.c - 1));
  p.nb = nseg * ((uint32_t)p.W << (p.c - 1));
  // chunks of <= K points (GBLS_MSM_K; measured r05: K = 8 fills the chip with ~1700 waves but
  // VALU busy stays at 0.43 -- the chunk loop waits on its point loads, not on SIMDs -- and the
  // larger folds cost 2.4 % of C2; K = 4 costs 5 %: K = 16 stays)
  p.K = g_msm_k;
  p.max_chunks = (uint32_t)(((uint64_t)p.W * n + p.K - 1) / p.K) + p.nb;
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
  const size_t tn = p.tree ? p.nb : 0;
  p.o_t0 = take(tn * sizeof(g2j));
  p.o_a0 = take(tn * sizeof(g2j));
  p.o_t1 = take((tn / 2 + 1) * sizeof(g2j));
  p.o_a1 = take((tn / 2 + 1) * sizeof(g2j));
  p.bytes = o;
  return p;
}

void launch_msm(hipStream_t st, const MsmPlan &p, uint8_t *ws, const g2a *sigs,
                const uint64_t *rands, const g1a *pks, const int32_t *pre, const int32_t *pre2,
                uint32_t n, const uint32_t *seg_off, int empty_is_error, g2a *H, g1s *P,
                int32_t *seg_err) {
  uint32_t *cnt = reinterpret_cast<uint32_t *>(ws + p.o_cnt);
  uint32_t *start = reinterpret_cast<uint32_t *>(ws + p.o_start);
  uint32_t *cur = reinterpret_cast<uint32_t *>(ws + p.o_cur);
  uint32_t *cstart = reinterpret_cast<uint32_t *>(ws + p.o_cstart);
  uint32_t *list = reinterpret_cast<uint32_t *>(ws + p.o_list);
  g2j *chunk = reinterpret_cast<g2j *>(ws + p.o_chunk);
  (void)hipMemsetAsync(cnt, 0, p.nb * 4, st);
  (void)hipMemsetAsync(seg_err, 0, p.nseg * 4, st);
  k_msm_count<<<nblk(n, WGR), WGR, 0, st>>>(sigs, rands, n, seg_off, p.nseg, p.c, p.W, pks, pre,
                                            pre2, cnt, seg_err);
  k_msm_scan<<<1, 1024, 0, st>>>(cnt, p.nb, p.K, start, cur, cstart);
  k_msm_scatter<<<nblk(n, WGR), WGR, 0, st>>>(sigs, rands, n, seg_off, p.nseg, p.c, p.W, cur,
                                              list);
  k_msm_chunk<<<nblk(p.max_chunks), WG, 0, st>>>(sigs, list, start, cstart, p.nb, p.max_chunks,
                                                 p.K, chunk);
  if (!p.tree) {
    k_msm_pairs<<<nblk(p.nb), WG, 0, st>>>(chunk, cstart, p.nb, p.extra, n, seg_off,
                                           empty_is_error, P, H, seg_err);
    return;
  }
  g2j *T[2] = {reinterpret_cast<g2j *>(ws + p.o_t0), reinterpret_cast<g2j *>(ws + p.o_t1)};
  g2j *A[2] = {reinterpret_cast<g2j *>(ws + p.o_a0), reinterpret_cast<g2j *>(ws + p.o_a1)};
  k_msm_bucket<<<nblk(p.nb), WG, 0, st>>>(chunk, cstart, p.nb, T[0], A[0]);
  int src = 0;
  const uint32_t B = 1u << (p.c - 1), groups = p.nseg * (uint32_t)p.W;
  for (int l = 0; (1u << (l + 1)) <= B; l++) {
    uint32_t m = B >> (l + 1);
    k_msm_tree<<<nblk((size_t)groups * m), WG, 0, st>>>(T[src], A[src], groups, m, l, T[1 - src],
                                                         A[1 - src]);
    src = 1 - src;
  }
  k_msm_wpairs<<<nblk(groups), WG, 0, st>>>(T[src], A[src], groups, (uint32_t)p.W, n, seg_off,
                                            empty_is_error, P, H, seg_err);
}

}  // namespace gbls
