// Device kernels of the MI355X BLS12-381 engine (gfx950).
//
// Layout in HBM: every per-set intermediate is an array-of-structures of 32-bit
// limbs (g1a 96 B, g2a 192 B, g2j 288 B, fp12 576 B).  One lane owns one set; a
// wave processes 64 consecutive sets, so each lane's 16-byte vector loads of its own
// element hit consecutive cache lines across the wave.  The work is VALU-integer
// bound (~10^6 mad64 per set against ~200 B of input), so the layout is chosen for
// simplicity of the per-lane code rather than for HBM bandwidth.
#pragma once
#include "bls_hash.h"
#include "bls_pairing.h"

namespace gbls {

constexpr int WG = 64;  // one wave per workgroup: the per-lane state is ~300 VGPRs

__device__ __constant__ uint8_t DST_POP[43] = {
    'B', 'L', 'S', '_', 'S', 'I', 'G', '_', 'B', 'L', 'S', '1', '2', '3', '8', '1',
    'G', '2', '_', 'X', 'M', 'D', ':', 'S', 'H', 'A', '-', '2', '5', '6', '_', 'S',
    'S', 'W', 'U', '_', 'R', 'O', '_', 'P', 'O', 'P', '_'};

__device__ __forceinline__ uint32_t gtid() { return blockIdx.x * blockDim.x + threadIdx.x; }

__device__ __forceinline__ void msg_ref(const uint8_t *data, const uint32_t *off, uint32_t i,
                                        const uint8_t *&p, uint32_t &len) {
  if (off) {
    p = data + off[i];
    len = off[i + 1] - off[i];
  } else {
    p = data + 32u * i;
    len = 32;
  }
}

// ---------------------------------------------------------------- decode / encode
__global__ void __launch_bounds__(WG) k_g1_decompress(const uint8_t *in, uint32_t n, int validate,
                                                      g1a *out, int32_t *st) {
  uint32_t i = gtid();
  if (i >= n) return;
  g1a a;
  int32_t s = g1_decompress(a, in + 48u * i);
  if (s == ST_SUCCESS && validate) {
    if (aff_is_inf(a))
      s = ST_PK_IS_INFINITY;
    else if (!g1_in_group(a))
      s = ST_NOT_IN_GROUP;
  }
  if (s != ST_SUCCESS) {
    fp_zero(a.x);
    fp_zero(a.y);
  }
  out[i] = a;
  st[i] = s;
}

__global__ void __launch_bounds__(WG) k_g2_decompress(const uint8_t *in, uint32_t n, g2a *out,
                                                      int32_t *st) {
  uint32_t i = gtid();
  if (i >= n) return;
  g2a a;
  int32_t s = g2_decompress(a, in + 96u * i);
  if (s != ST_SUCCESS) {
    fp2_zero(a.x);
    fp2_zero(a.y);
  }
  out[i] = a;
  st[i] = s;
}

__global__ void __launch_bounds__(WG) k_g2_validate(const g2a *in, uint32_t n, int32_t *st) {
  uint32_t i = gtid();
  if (i >= n) return;
  g2a a = in[i];
  st[i] = (g2_on_curve(a) || aff_is_inf(a)) && g2_in_group(a) ? ST_SUCCESS : ST_NOT_IN_GROUP;
}

__global__ void __launch_bounds__(WG) k_g1_compress(const g1a *in, uint32_t n, uint8_t *out) {
  uint32_t i = gtid();
  if (i >= n) return;
  g1_compress(out + 48u * i, in[i]);
}
__global__ void __launch_bounds__(WG) k_g2_compress(const g2a *in, uint32_t n, uint8_t *out) {
  uint32_t i = gtid();
  if (i >= n) return;
  g2_compress(out + 96u * i, in[i]);
}

// ---------------------------------------------------------------- segmented sums
// Workgroup reduction of one Jacobian point per lane through LDS (result in lane 0).
template <class F>
__device__ void wg_reduce_jac(jac<F> &v) {
  __shared__ jac<F> buf[WG];
  buf[threadIdx.x] = v;
  __syncthreads();
  for (int s = WG / 2; s > 0; s >>= 1) {
    if (threadIdx.x < (unsigned)s) {
      jac<F> o = buf[threadIdx.x + s];
      jac_add_n(v, v, o);
      buf[threadIdx.x] = v;
    }
    __syncthreads();
  }
}

// one workgroup per segment: pks[off[s] .. off[s+1]) -> affine sum (a4/a5)
__global__ void __launch_bounds__(WG) k_g1_aggregate_seg(const g1a *pks, const uint32_t *off,
                                                         uint32_t nseg, g1a *out, int32_t *st) {
  uint32_t s = blockIdx.x;
  if (s >= nseg) return;
  uint32_t b = off[s], e = off[s + 1];
  g1j acc;
  jac_set_inf(acc);
  for (uint32_t i = b + threadIdx.x; i < e; i += WG) jac_add_aff(acc, acc, pks[i]);
  wg_reduce_jac(acc);
  if (threadIdx.x == 0) {
    g1a r;
    jac_to_aff(r, acc);
    out[s] = r;
    st[s] = (e > b) ? ST_SUCCESS : ST_AGGR_TYPE_MISMATCH;
  }
}

__global__ void __launch_bounds__(WG) k_g2_aggregate_seg(const g2a *pts, const uint32_t *off,
                                                         uint32_t nseg, g2a *out) {
  uint32_t s = blockIdx.x;
  if (s >= nseg) return;
  uint32_t b = off[s], e = off[s + 1];
  g2j acc;
  jac_set_inf(acc);
  for (uint32_t i = b + threadIdx.x; i < e; i += WG) jac_add_aff(acc, acc, pts[i]);
  wg_reduce_jac(acc);
  if (threadIdx.x == 0) {
    g2a r;
    jac_to_aff(r, acc);
    out[s] = r;
  }
}

// ---------------------------------------------------------------- multi_verify stages
// H_i = hash_to_G2(m_i), affine
__global__ void __launch_bounds__(WG) k_hash_to_g2(const uint8_t *msg, const uint32_t *off,
                                                   uint32_t n, const uint8_t *dst, uint32_t dlen,
                                                   g2a *H) {
  uint32_t i = gtid();
  if (i >= n) return;
  const uint8_t *p;
  uint32_t len;
  msg_ref(msg, off, i, p, len);
  g2j h;
  hash_to_g2(h, p, len, dst_ref{dst ? dst : DST_POP, dst ? dlen : 43u});
  g2a a;
  jac_to_aff(a, h);
  H[i] = a;
}

// P_i = affine(r_i pk_i); bad_i = pk_i is infinity (blst PAIRING_Aggregate_PK_in_G1)
__global__ void __launch_bounds__(WG) k_mv_g1mul(const g1a *pks, const uint64_t *rands, uint32_t n,
                                                 g1a *P, int32_t *bad) {
  uint32_t i = gtid();
  if (i >= n) return;
  g1a pk = pks[i];
  g1j t;
  mul_u64(t, pk, rands[i]);
  g1a a;
  jac_to_aff(a, t);
  P[i] = a;
  bad[i] = aff_is_inf(pk) ? 1 : 0;
}

// R_i = r_i sig_i (Jacobian); infinite signatures contribute the identity
__global__ void __launch_bounds__(WG) k_mv_g2mul(const g2a *sigs, const uint64_t *rands, uint32_t n,
                                                 g2j *R) {
  uint32_t i = gtid();
  if (i >= n) return;
  g2j t;
  mul_u64(t, sigs[i], rands[i]);
  R[i] = t;
}

// S_s = sum of R_i over segment s (one workgroup per segment)
__global__ void __launch_bounds__(WG) k_seg_g2_sum(const g2j *R, const uint32_t *off,
                                                   uint32_t nseg, g2j *S) {
  uint32_t s = blockIdx.x;
  if (s >= nseg) return;
  g2j acc;
  jac_set_inf(acc);
  for (uint32_t i = off[s] + threadIdx.x; i < off[s + 1]; i += WG) jac_add_n(acc, acc, R[i]);
  wg_reduce_jac(acc);
  if (threadIdx.x == 0) S[s] = acc;
}

// f_i = MillerLoop(P_i, H_i)
__global__ void __launch_bounds__(WG) k_miller(const g1a *P, const g2a *H, uint32_t n, fp12 *f) {
  uint32_t i = gtid();
  if (i >= n) return;
  fp12 r;
  miller_loop(r, P[i], H[i]);
  f[i] = r;
}

// F_s = prod f_i over segment s; err_s = OR of bad_i (one workgroup per segment)
__global__ void __launch_bounds__(WG) k_seg_fp12_prod(const fp12 *f, const int32_t *bad,
                                                      const uint32_t *off, uint32_t nseg,
                                                      fp12 *F, int32_t *err) {
  __shared__ int32_t e_sh;
  uint32_t s = blockIdx.x;
  if (s >= nseg) return;
  if (threadIdx.x == 0) e_sh = 0;
  __syncthreads();
  fp12 acc;
  fp12_one(acc);
  int32_t e = 0;
  for (uint32_t i = off[s] + threadIdx.x; i < off[s + 1]; i += WG) {
    fp12_mul_n(acc, acc, f[i]);
    e |= bad[i];
  }
  if (e) atomicOr(&e_sh, 1);
  // tree product through LDS, 16 lanes at a time to bound LDS use (576 B per element)
  __shared__ fp12 buf[16];
  for (int base = 16; base < WG; base += 16) {
    __syncthreads();
    if (threadIdx.x >= (unsigned)base && threadIdx.x < (unsigned)base + 16)
      buf[threadIdx.x - base] = acc;
    __syncthreads();
    if (threadIdx.x < 16) fp12_mul_n(acc, acc, buf[threadIdx.x]);
  }
  for (int w = 8; w > 0; w >>= 1) {
    __syncthreads();
    if (threadIdx.x >= (unsigned)w && threadIdx.x < (unsigned)2 * w) buf[threadIdx.x - w] = acc;
    __syncthreads();
    if (threadIdx.x < (unsigned)w) fp12_mul_n(acc, acc, buf[threadIdx.x]);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    F[s] = acc;
    err[s] = e_sh | (off[s + 1] == off[s] ? 1 : 0);
  }
}

// partial_s = F_s * MillerLoop(-g1, S_s)   (the segment's own e(-g1, sum r sig) term)
__global__ void __launch_bounds__(WG) k_seg_partial(const fp12 *F, const g2j *S, uint32_t nseg,
                                                    fp12 *part) {
  uint32_t s = gtid();
  if (s >= nseg) return;
  g2a sa;
  jac_to_aff(sa, S[s]);
  g1a ng1;
  fp_set(ng1.x, k::G1X_M);
  fp_set(ng1.y, k::G1NEGY_M);
  fp12 m;
  miller_loop(m, ng1, sa);
  fp12 r;
  fp12_mul_n(r, F[s], m);
  part[s] = r;
}

// verdict_s = FE(prod_k partial[k][s]) == 1 and no segment error on any part
__global__ void __launch_bounds__(WG) k_final_verify(const fp12 *part, const int32_t *err,
                                                     uint32_t nparts, uint32_t nseg,
                                                     int32_t *verdict) {
  uint32_t s = gtid();
  if (s >= nseg) return;
  fp12 acc = part[s];
  int32_t e = err[s];
  for (uint32_t k = 1; k < nparts; k++) {
    fp12_mul_n(acc, acc, part[(size_t)k * nseg + s]);
    e |= err[(size_t)k * nseg + s];
  }
  fp12 r;
  final_exp(r, acc);
  verdict[s] = (!e && fp12_is_one(r)) ? ST_SUCCESS : ST_VERIFY_FAIL;
}

// ---------------------------------------------------------------- single-pair checks
// f_i = ML(pk_i, H_i) * ML(-g1, sig_i) with blst's pre-checks (a6/a7):
// infinite pk -> fail; sig must be in G2 (sig_groupcheck = true); infinite sig skipped.
__global__ void __launch_bounds__(WG) k_av_miller(const g2a *sigs, const g1a *pks, const g2a *H,
                                                  const int32_t *pre, uint32_t m, fp12 *f,
                                                  int32_t *bad) {
  uint32_t i = gtid();
  if (i >= m) return;
  g1a pk = pks[i];
  g2a sig = sigs[i];
  int32_t b = (pre && pre[i] != ST_SUCCESS) ? 1 : 0;
  if (aff_is_inf(pk)) b = 1;
  if (!aff_is_inf(sig) && !g2_in_group(sig)) b = 1;
  fp12 r;
  fp12_one(r);
  if (!b) {
    miller_loop(r, pk, H[i]);
    if (!aff_is_inf(sig)) {
      g1a ng1;
      fp_set(ng1.x, k::G1X_M);
      fp_set(ng1.y, k::G1NEGY_M);
      fp12 t;
      miller_loop(t, ng1, sig);
      fp12_mul_n(r, r, t);
    }
  }
  f[i] = r;
  bad[i] = b;
}

// ---------------------------------------------------------------- key material (a15)
HD void scalar_from_be32(uint32_t (&s)[8], const uint8_t *b) {
  for (int i = 0; i < 8; i++) {
    const uint8_t *q = b + 4 * (7 - i);
    s[i] = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | q[3];
  }
}
template <class F>
__device__ void mul_scalar256(jac<F> &r, const aff<F> &base, const uint32_t (&s)[8]) {
  jac<F> acc;
  jac_set_inf(acc);
  for (int i = 255; i >= 0; i--) {
    jac_dbl(acc, acc);
    if ((s[i >> 5] >> (i & 31)) & 1) jac_add_aff(acc, acc, base);
  }
  r = acc;
}

__global__ void __launch_bounds__(WG) k_sk_to_pk(const uint8_t *sks, uint32_t n, g1a *out) {
  uint32_t i = gtid();
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
  uint32_t i = gtid();
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
// 8 independent v_mad_u64_u32 chains per lane; returns nothing useful, the timing is
// the measurement (2 * iters * 8 mads per lane).
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

}  // namespace gbls
