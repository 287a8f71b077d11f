// gfx950 kernels: segmented point aggregation (a4, a5, a11: one 256-lane workgroup per
// segment), key material for fixtures (a15) and the v_mad_u64_u32 roofline probe.
#include "gbls_common.h"
#include "bls_w4.h"

namespace gbls {

// Workgroup tree reduction of one Jacobian point per lane through LDS (result: lane 0)
template <class F>
__device__ __forceinline__ void wg_reduce_jac(jac<F> &v) {
  __shared__ jac<F> buf[WGR / 2];
  for (int w = WGR / 2; w > 0; w >>= 1) {
    __syncthreads();
    if (threadIdx.x >= (unsigned)w && threadIdx.x < (unsigned)2 * w) buf[threadIdx.x - w] = v;
    __syncthreads();
    if (threadIdx.x < (unsigned)w) {
      jac<F> o = buf[threadIdx.x];
      jac_add(v, v, o);
    }
  }
}

// one workgroup per segment: pks[off[s] .. off[s+1]) -> affine sum (a4/a5)
__global__ void __launch_bounds__(WGR) k_g1_aggregate_seg(const g1a *pks, const uint32_t *off,
                                                          uint32_t nseg, g1a *out, int32_t *st) {
  uint32_t s = blockIdx.x;
  if (s >= nseg) return;
  uint32_t b = off[s], e = off[s + 1];
  g1j acc;
  jac_set_inf(acc);
  for (uint32_t i = b + threadIdx.x; i < e; i += WGR) jac_add_aff(acc, acc, pks[i]);
  wg_reduce_jac(acc);
  if (threadIdx.x == 0) {
    g1a r;
    jac_to_aff(r, acc);
    out[s] = r;
    st[s] = (e > b) ? ST_SUCCESS : ST_AGGR_TYPE_MISMATCH;
  }
}

__global__ void __launch_bounds__(WGR) k_g2_aggregate_seg(const g2a *pts, const uint32_t *off,
                                                          uint32_t nseg, g2a *out, int32_t *st) {
  uint32_t s = blockIdx.x;
  if (s >= nseg) return;
  uint32_t b = off[s], e = off[s + 1];
  g2j acc;
  jac_set_inf(acc);
  for (uint32_t i = b + threadIdx.x; i < e; i += WGR) jac_add_aff(acc, acc, pts[i]);
  wg_reduce_jac(acc);
  if (threadIdx.x == 0) {
    g2a r;
    jac_to_aff(r, acc);
    out[s] = r;
    if (st) st[s] = (e > b) ? ST_SUCCESS : ST_AGGR_TYPE_MISMATCH;
  }
}

// ---------------------------------------------------------------- validator registry (f1)
// Public keys addressed by validator index into a device-resident table of decompressed,
// validated keys (the CachedPublicKey cache, bls/src/cached_public_key.rs:104-108, one
// per Validator.pubkey, types/src/phase0/containers.rs:229).  Invalid keys and slots never
// loaded are stored all-zero (infinity).  A valid key is never infinity (PublicKey::try_from
// validates, bls/src/public_key.rs:20-28), so every gather below flags an all-zero entry
// BAD_ENCODING like an out-of-range index: the reference fails the whole check when one
// member key does not decompress (helper_functions/src/predicates.rs:130).

// one workgroup per segment: sum of reg[idx[off[s] .. off[s+1])] (Triple::verify_aggregate,
// helper_functions/src/verifier.rs:387-405); st = AGGR_TYPE_MISMATCH when empty,
// BAD_ENCODING when an index is out of range or names an invalid / unloaded (all-zero)
// entry.  An infinite sum of valid keys is a SUCCESS (as in AggregatePublicKey::aggregate);
// the verification paths reject infinite keys.
__global__ void __launch_bounds__(WGR) k_g1_aggregate_idx(const g1a *reg, uint32_t nreg,
                                                          const uint32_t *idx, const uint32_t *off,
                                                          uint32_t nseg, g1a *out, int32_t *st) {
  __shared__ int32_t oob_sh;
  uint32_t s = blockIdx.x;
  if (s >= nseg) return;
  if (threadIdx.x == 0) oob_sh = 0;
  __syncthreads();
  uint32_t b = off[s], e = off[s + 1];
  g1j acc;
  jac_set_inf(acc);
  int32_t oob = 0;
  for (uint32_t i = b + threadIdx.x; i < e; i += WGR) {
    uint32_t v = idx[i];
    if (v < nreg && !aff_is_inf(reg[v]))
      jac_add_aff(acc, acc, reg[v]);
    else
      oob = 1;
  }
  if (oob) atomicOr(&oob_sh, 1);
  wg_reduce_jac(acc);
  if (threadIdx.x == 0) {
    g1a r;
    jac_to_aff(r, acc);
    int32_t status = ST_SUCCESS;
    if (e == b)
      status = ST_AGGR_TYPE_MISMATCH;
    else if (oob_sh)
      status = ST_BAD_ENCODING;
    if (status != ST_SUCCESS) {
      fp_zero(r.x);
      fp_zero(r.y);
    }
    out[s] = r;
    st[s] = status;
  }
}

// one key per set: out[i] = reg[idx[i]] (all-zero + BAD_ENCODING when out of range or
// the entry is invalid / unloaded)
__global__ void __launch_bounds__(WG) k_g1_gather_idx(const g1a *reg, uint32_t nreg,
                                                      const uint32_t *idx, uint32_t n, g1a *out,
                                                      int32_t *st) {
  uint32_t i = blockIdx.x * WG + threadIdx.x;
  if (i >= n) return;
  uint32_t v = idx[i];
  g1a r;
  bool ok = v < nreg;
  if (ok) {
    r = reg[v];
    ok = !aff_is_inf(r);
  } else {
    fp_zero(r.x);
    fp_zero(r.y);
  }
  out[i] = r;
  st[i] = ok ? ST_SUCCESS : ST_BAD_ENCODING;
}

// ---------------------------------------------------------------- row aggregation
// Many segments (committees, sync-committee messages): one DPP row (16 lanes) per
// segment instead of a 256-lane workgroup.  Each lane sums every 16th key with mixed
// additions, the row folds its 16 partial sums in 4 row_shl steps (VALU moves, no LDS,
// no barrier), and the row's lane 0 converts to affine: four segments per wave share
// one inversion's latency, where the workgroup form spends a tree of 8 LDS levels and a
// whole inversion per segment.
template <int K>
__device__ __forceinline__ uint32_t row_shl(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x100 + K, 0xf, 0xf, true);
}
template <int K, class F>
__device__ __forceinline__ void jac_row_fold(jac<F> &acc, uint32_t &flag) {
  jac<F> o;
  uint32_t *d = reinterpret_cast<uint32_t *>(&o);
  const uint32_t *a = reinterpret_cast<const uint32_t *>(&acc);
#pragma unroll
  for (int i = 0; i < (int)(sizeof(jac<F>) / 4); i++) d[i] = row_shl<K>(a[i]);
  flag |= row_shl<K>(flag);
  jac_add(acc, acc, o);  // lanes past the row end read zeros: infinity
}
// segment s = sum of pts[i] (idx == nullptr) or reg[idx[i]], i in [off[s], off[s+1])
template <class F, bool X>
__global__ void __launch_bounds__(WG) k_aggregate_rows(const aff<F> *pts, uint32_t nreg,
                                                       const uint32_t *idx, const uint32_t *off,
                                                       uint32_t nseg, aff<F> *out, int32_t *st) {
  if constexpr (X) w4::exclusive_simd();
  uint32_t t = blockIdx.x * WG + threadIdx.x;
  uint32_t s = t >> 4, r = t & 15;
  if (s >= nseg) return;  // whole rows
  uint32_t b = off[s], e = off[s + 1];
  jac<F> acc;
  jac_set_inf(acc);
  uint32_t oob = 0;
  for (uint32_t i = b + r; i < e; i += 16) {
    uint32_t v = idx ? idx[i] : i;
    if (idx && (v >= nreg || aff_is_inf(pts[v])))  // registry: out of range / invalid slot
      oob = 1;
    else
      jac_add_aff(acc, acc, pts[v]);
  }
  jac_row_fold<1>(acc, oob);
  jac_row_fold<2>(acc, oob);
  jac_row_fold<4>(acc, oob);
  jac_row_fold<8>(acc, oob);
  if (r != 0) return;
  aff<F> o;
  jac_to_aff(o, acc);
  int32_t status = ST_SUCCESS;
  if (e == b)
    status = ST_AGGR_TYPE_MISMATCH;
  else if (oob)
    status = ST_BAD_ENCODING;
  if (idx && status != ST_SUCCESS) {
    f_zero(o.x);
    f_zero(o.y);
  }
  out[s] = o;
  if (st) st[s] = status;
}
// rows for many segments; the 256-lane workgroup form for a few long ones
constexpr uint32_t kRowAggregateMinSegs = 128;

// ---------------------------------------------------------------- key material (a15)
HD void scalar_from_be32(uint32_t (&s)[8], const uint8_t *b) {
  for (int i = 0; i < 8; i++) {
    const uint8_t *q = b + 4 * (7 - i);
    s[i] = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | q[3];
  }
}
template <class F>
__device__ __forceinline__ void mul_scalar256(jac<F> &r, const aff<F> &base, const uint32_t (&s)[8]) {
  jac<F> acc;
  jac_set_inf(acc);
  for (int i = 255; i >= 0; i--) {
    jac_dbl(acc, acc);
    if ((s[i >> 5] >> (i & 31)) & 1) jac_add_aff(acc, acc, base);
  }
  r = acc;
}

__global__ void __launch_bounds__(WG) k_sk_to_pk(const uint8_t *sks, uint32_t n, g1a *out) {
  uint32_t i = blockIdx.x * WG + threadIdx.x;
  if (i >= n) return;
  uint32_t s[8];
  scalar_from_be32(s, sks + 32u * i);
  g1a g;
  fp_set(g.x, k::G1X_M);
  fp_set(g.y, k::G1Y_M);
  g1j t;
  mul_scalar256(t, g, s);
  g1a a;
  jac_to_aff(a, t);
  out[i] = a;
}

__global__ void __launch_bounds__(WG) k_sign(const uint8_t *sks, const g2a *H, uint32_t n,
                                             g2a *out) {
  uint32_t i = blockIdx.x * WG + threadIdx.x;
  if (i >= n) return;
  uint32_t s[8];
  scalar_from_be32(s, sks + 32u * i);
  g2j t;
  mul_scalar256(t, H[i], s);
  g2a a;
  jac_to_aff(a, t);
  out[i] = a;
}

// ---------------------------------------------------------------- roofline probe
// 8 independent v_mad_u64_u32 chains per lane (2 * iters * 8 mads per lane)
__global__ void __launch_bounds__(256) k_mad_peak(uint64_t *sink, uint32_t iters, uint32_t seed) {
  uint32_t a = seed ^ threadIdx.x, b = seed * 2654435761u + blockIdx.x;
  uint64_t acc[8];
#pragma unroll
  for (int j = 0; j < 8; j++) acc[j] = (uint64_t)(a + j) << 7;
  for (uint32_t it = 0; it < iters; it++) {
#pragma unroll
    for (int j = 0; j < 8; j++) acc[j] = (uint64_t)(uint32_t)acc[j] * b + acc[j];
#pragma unroll
    for (int j = 0; j < 8; j++) acc[j] = (uint64_t)(uint32_t)(acc[j] >> 32) * a + acc[j];
  }
  uint64_t x = 0;
#pragma unroll
  for (int j = 0; j < 8; j++) x ^= acc[j];
  if (x == 0x123456789ull) sink[0] = x;
}

// ---------------------------------------------------------------- launchers
void launch_g1_aggregate_seg(hipStream_t st, const g1a *pks, const uint32_t *off, uint32_t nseg,
                             g1a *out, int32_t *status) {
  if (nseg >= kRowAggregateMinSegs)
    (nblk(16 * (size_t)nseg) <= w4::kExclusiveMaxWaves ? k_aggregate_rows<fp, true> : k_aggregate_rows<fp, false>)<<<nblk(16 * (size_t)nseg), WG, 0, st>>>(pks, 0, nullptr, off, nseg, out,
                                                                 status);
  else if (nseg)
    k_g1_aggregate_seg<<<nseg, WGR, 0, st>>>(pks, off, nseg, out, status);
}
void launch_g2_aggregate_seg(hipStream_t st, const g2a *pts, const uint32_t *off, uint32_t nseg,
                             g2a *out, int32_t *status) {
  if (nseg >= kRowAggregateMinSegs)
    (nblk(16 * (size_t)nseg) <= w4::kExclusiveMaxWaves ? k_aggregate_rows<fp2, true> : k_aggregate_rows<fp2, false>)<<<nblk(16 * (size_t)nseg), WG, 0, st>>>(pts, 0, nullptr, off, nseg, out,
                                                                  status);
  else if (nseg)
    k_g2_aggregate_seg<<<nseg, WGR, 0, st>>>(pts, off, nseg, out, status);
}
void launch_g1_aggregate_idx(hipStream_t st, const g1a *reg, uint32_t nreg, const uint32_t *idx,
                             const uint32_t *off, uint32_t nseg, g1a *out, int32_t *status) {
  if (nseg >= kRowAggregateMinSegs)
    (nblk(16 * (size_t)nseg) <= w4::kExclusiveMaxWaves ? k_aggregate_rows<fp, true> : k_aggregate_rows<fp, false>)<<<nblk(16 * (size_t)nseg), WG, 0, st>>>(reg, nreg, idx, off, nseg, out,
                                                                 status);
  else if (nseg)
    k_g1_aggregate_idx<<<nseg, WGR, 0, st>>>(reg, nreg, idx, off, nseg, out, status);
}
void launch_g1_gather_idx(hipStream_t st, const g1a *reg, uint32_t nreg, const uint32_t *idx,
                          uint32_t n, g1a *out, int32_t *status) {
  if (n) k_g1_gather_idx<<<nblk(n), WG, 0, st>>>(reg, nreg, idx, n, out, status);
}
void launch_sk_to_pk(hipStream_t st, const uint8_t *sks, uint32_t n, g1a *out) {
  if (n) k_sk_to_pk<<<nblk(n), WG, 0, st>>>(sks, n, out);
}
void launch_sign(hipStream_t st, const uint8_t *sks, const g2a *H, uint32_t n, g2a *out) {
  if (n) k_sign<<<nblk(n), WG, 0, st>>>(sks, H, n, out);
}
void launch_mad_peak(hipStream_t st, unsigned blocks, uint64_t *sink, uint32_t iters, uint32_t seed) {
  k_mad_peak<<<blocks, 256, 0, st>>>(sink, iters, seed);
}

}  // namespace gbls
