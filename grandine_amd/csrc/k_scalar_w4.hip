// gfx950 kernels: the wave-per-point (W4, bls_w4.h) forms of the random-scalar products and of
// the per-segment signature sum -- the latency regime of k_scalar.hip's stages (launches of
// <= kW4Max points), in a translation unit of their own so that the two compile in parallel.
#include "gbls_common.h"
#include "bls_w4.h"

namespace gbls {

// P_i = r_i pk_i, one wave per set (bls_w4.h dbl1 / madd1: three rounds per doubling, six
// per addition), written as the line-evaluation point (X Z, Y, Z^3) -- the latency regime
template <bool X>
__global__ void __launch_bounds__(64) k_mv_g1mul_w4(const g1a *pks, const uint64_t *rands, uint32_t n,
                                                    g1s *P) {
  if constexpr (X) w4::exclusive_simd();
  const uint32_t i = blockIdx.x;
  if (i >= n) return;  // whole waves
  const g1a pk = pks[i];
  const uint64_t k = rands[i];
  const uint32_t j = threadIdx.x & 15, r = (threadIdx.x >> 4) & 3;
  if (k == 0 || aff_is_inf(pk)) {  // g1s_from_jac of infinity: all zero
    if (j < 12 && r == 0) {
      P[i].x.l[j] = 0;
      P[i].y.l[j] = 0;
      P[i].c.l[j] = 0;
    }
    return;
  }
  w4::Ctx c;
  w4::init(c);
  const uint32_t cin = dfp::konst(dfp::K_CIN);
  uint32_t x2, y2, d0, d1;
  w4::mul4(c, x2, y2, d0, d1, w4::repack(pk.x, j), cin, w4::repack(pk.y, j), cin, w4::repack(pk.x, j), cin,
           w4::repack(pk.y, j), cin);
  w4::J1 acc{x2, y2, c.one};
  const int top = 63 - __clzll((long long)k);
  for (int bit = top - 1; bit >= 0; bit--) {
    w4::dbl1(c, acc, acc);
    if ((k >> bit) & 1) w4::madd1(c, acc, acc, x2, y2);
  }
  // (X Z, Y, Z^3): Z = 0 (infinity) gives all-zero x and c, as g1s_from_jac
  uint32_t xz, z2;
  w4::mul4(c, xz, z2, d0, d1, acc.x, acc.z, acc.z, acc.z, acc.x, acc.z, acc.x, acc.z);
  uint32_t z3;
  w4::mul4(c, z3, d0, d1, d1, z2, acc.z, z2, acc.z, z2, acc.z, z2, acc.z);
  const uint32_t w = dfp::word_of(w4::sel(c, xz, acc.y, z3, z3), c.t);
  if (j < 12 && r == 0) P[i].x.l[j] = w;
  if (j < 12 && r == 1) P[i].y.l[j] = w;
  if (j < 12 && r == 2) P[i].c.l[j] = w;
}

// the same halves, one wave per (set, half) (bls_w4.h): a doubling is four rounds of four
// row-distributed products, a mixed addition eight -- the latency regime
template <bool X>
__global__ void __launch_bounds__(64) k_mv_g2mul_w4(const g2a *sigs, const uint64_t *rands,
                                                    uint32_t n, g2j *R) {
  if constexpr (X) w4::exclusive_simd();
  const uint32_t t = blockIdx.x;
  if (t >= 2 * n) return;  // whole waves
  const uint32_t i = t < n ? t : t - n;
  const uint64_t r = rands ? rands[i] : 1;
  const uint64_t k = t < n ? (r & 0xffffffffull) : (r >> 32);
  const g2a base = sigs[i];
  const uint32_t j = threadIdx.x & 15;
  if (k == 0 || aff_is_inf(base)) {  // identity (jac_set_inf)
    if (threadIdx.x < 12) {
      uint32_t one = 0;
#pragma unroll
      for (int q = 0; q < 12; q++) one = j == (uint32_t)q ? k::ONE_M[q] : one;
      R[t].x.c0.l[j] = one;
      R[t].x.c1.l[j] = 0;
      R[t].y.c0.l[j] = one;
      R[t].y.c1.l[j] = 0;
      R[t].z.c0.l[j] = 0;
      R[t].z.c1.l[j] = 0;
    }
    return;
  }
  w4::Ctx c;
  w4::init(c);
  w4::A2 b;
  w4::load(c, b, base);
  w4::J acc;
  acc.x = b.x;
  acc.y = b.y;
  acc.z = {c.one, 0u};
  const int top = 63 - __clzll((long long)k);
  for (int bit = top - 1; bit >= 0; bit--) {
    w4::dbl(c, acc, acc);
    if ((k >> bit) & 1) w4::madd(c, acc, acc, b);
  }
  w4::store_jac(c, R + t, acc);
}

// level 2 on one workgroup of kFinalW4Waves waves per segment (bls_w4.h, one wave per SIMD):
// wave w sums the segment's chunk partials q = w, w + NW, ... (a low- and a high-half
// accumulator), a two-level tree joins the waves through LDS (the row-form registers as they
// are), then wave 0 applies the 2^32 shift of the high half (32 doublings) and stores S --
// ~0.3 ms instead of the quads' ~0.6 ms (their one-lane inversion dominates).  The serial
// additions over the chunk partials drop from one per chunk (16 for a 2048-set segment) to
// ceil(chunks / NW) + 2 per half: the signature side sets the join of C4-shaped submissions
// (profiles/r06/zz_c4_join_wait.txt).  S is the same group element (only its Jacobian scale
// changes, which the final exponentiation removes from its lines).
constexpr int kFinalW4Waves = 4;
template <bool X>
__global__ void __launch_bounds__(64 * kFinalW4Waves) k_g2sum_final_w4(const g2j *part, const int32_t *part_err,
                                                                       const uint32_t *chunks, const uint32_t *seg_chunk,
                                                                       const uint32_t *seg_off, uint32_t nseg, uint32_t n,
                                                                       int empty_is_error, g1s *P, g2a *H,
                                                                       int32_t *seg_err, g2j *Sj) {
  if constexpr (X) w4::exclusive_simd();
  constexpr int NW = kFinalW4Waves;
  __shared__ uint32_t sh[NW / 2][12 * 64];  // a sending wave's lo and hi, word k of lane l at k * 64 + l
  __shared__ int32_t sh_err[NW];
  const uint32_t s = blockIdx.x;
  if (s >= nseg) return;  // block-uniform
  const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  w4::Ctx c;
  w4::init(c);
  w4::J lo, hi;
  w4::set_inf(c, lo);
  w4::set_inf(c, hi);
  int32_t err = 0;
  for (uint32_t q = seg_chunk[s] + w; q < seg_chunk[s + 1]; q += NW) {
    w4::J v;
    w4::load(c, v, part[q]);
    if (chunks[4 * q + 1] == 0)
      w4::add(c, lo, lo, v);
    else
      w4::add(c, hi, hi, v);
    err |= part_err[q];
  }
  if (lane == 0) sh_err[w] = err;
  for (uint32_t width = NW / 2; width > 0; width >>= 1) {
    __syncthreads();
    if (w >= width && w < 2 * width) {
      uint32_t *d = sh[w - width] + lane;
      const uint32_t v[12] = {lo.x.c0, lo.x.c1, lo.y.c0, lo.y.c1, lo.z.c0, lo.z.c1,
                              hi.x.c0, hi.x.c1, hi.y.c0, hi.y.c1, hi.z.c0, hi.z.c1};
#pragma unroll
      for (int k = 0; k < 12; k++) d[64 * k] = v[k];
    }
    __syncthreads();
    if (w < width) {
      const uint32_t *d = sh[w] + lane;
      w4::J o;
      o.x = {d[0], d[64]};
      o.y = {d[128], d[192]};
      o.z = {d[256], d[320]};
      w4::add(c, lo, lo, o);
      o.x = {d[384], d[448]};
      o.y = {d[512], d[576]};
      o.z = {d[640], d[704]};
      w4::add(c, hi, hi, o);
    }
  }
  if (w != 0) return;  // wave-uniform; no barrier follows
#pragma unroll
  for (int k = 1; k < NW; k++) err |= sh_err[k];
  if (empty_is_error && seg_off[s + 1] == seg_off[s]) err = 1;
  for (int d = 0; d < 32; d++) w4::dbl(c, hi, hi);
  w4::add(c, lo, lo, hi);
  if (Sj)
    w4::store_jac(c, Sj + s, lo);  // the lines take it projectively (k_lines_w4j)
  else
    w4::store_affine(c, H + n + s, lo);
  if (threadIdx.x == 0) {
    g1s ng1;
    fp_set(ng1.x, k::G1X_M);
    fp_set(ng1.y, k::G1NEGY_M);
    fp_one(ng1.c);
    P[n + s] = ng1;
    seg_err[s] = err;
  }
}

void launch_mv_g1mul_w4(hipStream_t st, const g1a *pks, const uint64_t *rands, uint32_t n, g1s *P) {
  (n <= w4::kExclusiveMaxWaves ? k_mv_g1mul_w4<true> : k_mv_g1mul_w4<false>)<<<n, 64, 0, st>>>(pks, rands, n, P);
}
void launch_mv_g2mul_w4(hipStream_t st, const g2a *sigs, const uint64_t *rands, uint32_t n, g2j *R) {
  (2 * n <= w4::kExclusiveMaxWaves ? k_mv_g2mul_w4<true> : k_mv_g2mul_w4<false>)<<<2 * n, 64, 0, st>>>(sigs, rands,
                                                                                                     n, R);
}
void launch_g2sum_final_w4(hipStream_t st, const g2j *part, const int32_t *part_err, const uint32_t *chunks,
                           const uint32_t *seg_chunk, const uint32_t *seg_off, uint32_t nseg, uint32_t n,
                           int empty_is_error, g1s *P, g2a *H, int32_t *seg_err, g2j *Sj) {
  (nseg * kFinalW4Waves <= w4::kExclusiveMaxWaves ? k_g2sum_final_w4<true> : k_g2sum_final_w4<false>)<<<
      nseg, 64 * kFinalW4Waves, 0, st>>>(part, part_err, chunks, seg_chunk, seg_off, nseg, n, empty_is_error, P, H,
                                         seg_err, Sj);
}

}  // namespace gbls
