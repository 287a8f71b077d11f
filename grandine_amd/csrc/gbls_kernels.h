// Device kernels of the MI355X BLS12-381 engine (gfx950).
//
// Execution model: one lane owns one signature set (or one hash-to-field element,
// or one segment for the reductions).  All field arithmetic is inlined into small
// stage kernels -- each stage keeps its working set (<= ~3 Fp12 values plus
// temporaries) in the unified 512-entry VGPR/AGPR file at one wave per SIMD, and
// hands its result to the next stage through HBM.
//
// Layout in HBM: per-set intermediates are arrays of structures of 32-bit limbs
// (g1p 144 B, g2h 288 B, g2j 288 B, fp12 576 B).  A set needs ~10^6 mad64 against
// ~2 KB of intermediate traffic, so the stages are VALU bound and the layout is
// chosen for simple per-lane code, not for bandwidth (roofline).
#pragma once
#include "bls_hash.h"
#include "bls_pairing.h"

namespace gbls {

constexpr int WG = 64;    // per-lane kernels: one wave per workgroup
constexpr int WGR = 256;  // segment reductions: 4 waves, LDS tree

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

__device__ __forceinline__ void neg_g1_gen(g1a &a) {
  fp_set(a.x, k::G1X_M);
  fp_set(a.y, k::G1NEGY_M);
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

// signature subgroup check (sig_groupcheck = true in verify / fast_aggregate_verify);
// infinity passes.  st[i] |= 1 on failure when `accumulate`, else st[i] = status.
__global__ void __launch_bounds__(WG) k_g2_check(const g2a *in, uint32_t n, int32_t *st,
                                                 int accumulate) {
  uint32_t i = gtid();
  if (i >= n) return;
  g2a a = in[i];
  bool ok = aff_is_inf(a) || (g2_on_curve(a) && g2_in_group(a));
  if (accumulate)
    st[i] = st[i] | (ok ? 0 : 1);
  else
    st[i] = ok ? ST_SUCCESS : ST_NOT_IN_GROUP;
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
// Workgroup tree reduction of one Jacobian point per lane through LDS (result: lane 0)
template <class F>
__device__ void wg_reduce_jac(jac<F> &v) {
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
                                                          uint32_t nseg, g2a *out) {
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
  }
}

// ---------------------------------------------------------------- hash_to_G2 stages
// stage 1: expand_message_xmd + hash_to_field -> u[0], u[1]
__global__ void __launch_bounds__(WG) k_h2c_field(const uint8_t *msg, const uint32_t *off,
                                                  uint32_t n, const uint8_t *dst, uint32_t dlen,
                                                  fp2 *U) {
  uint32_t i = gtid();
  if (i >= n) return;
  const uint8_t *p;
  uint32_t len;
  msg_ref(msg, off, i, p, len);
  fp2 u[2];
  hash_to_field_g2(u, p, len, dst_ref{dst ? dst : DST_POP, dst ? dlen : 43u});
  U[2 * i] = u[0];
  U[2 * i + 1] = u[1];
}
// stage 2: one lane per field element: SSWU on E2' + 3-isogeny -> Jacobian on E2
__global__ void __launch_bounds__(WG) k_h2c_map(const fp2 *U, uint32_t nu, g2j *Q) {
  uint32_t i = gtid();
  if (i >= nu) return;
  g2j q;
  map_to_g2(q, U[i]);
  Q[i] = q;
}
// stage 3: Q0 + Q1, clear cofactor -> homogeneous projective H (Miller-loop input)
__global__ void __launch_bounds__(WG) k_h2c_clear(const g2j *Q, uint32_t n, g2h *H) {
  uint32_t i = gtid();
  if (i >= n) return;
  g2j a = Q[2 * i], b = Q[2 * i + 1], h;
  jac_add(a, a, b);
  clear_cofactor_g2(h, a);
  g2h o;
  g2h_from_jac(o, h);
  H[i] = o;
}
// homogeneous -> affine (API outputs, signing)
__global__ void __launch_bounds__(WG) k_g2h_to_aff(const g2h *H, uint32_t n, g2a *out) {
  uint32_t i = gtid();
  if (i >= n) return;
  g2h h = H[i];
  g2a a;
  if (fp2_is_zero(h.z)) {
    fp2_zero(a.x);
    fp2_zero(a.y);
  } else {
    fp2 zi;
    fp2_inv(zi, h.z);
    fp2_mul(a.x, h.x, zi);
    fp2_mul(a.y, h.y, zi);
  }
  out[i] = a;
}

// ---------------------------------------------------------------- batch-verify stages
// P_i = r_i pk_i in Miller form; bad_i = pk infinite (blst PAIRING_Aggregate_PK_in_G1)
// or a caller pre-check failed (signature subgroup check, aggregation status).
__global__ void __launch_bounds__(WG) k_mv_g1mul(const g1a *pks, const uint64_t *rands,
                                                 const int32_t *pre, uint32_t n, g1p *P,
                                                 int32_t *bad) {
  uint32_t i = gtid();
  if (i >= n) return;
  g1a pk = pks[i];
  uint64_t r = rands ? rands[i] : 1;
  g1j t;
  mul_u64(t, pk, r);
  g1p o;
  g1p_from_jac(o, t);
  P[i] = o;
  bad[i] = (aff_is_inf(pk) || (pre && pre[i] != 0)) ? 1 : 0;
}

// R_i = r_i sig_i (Jacobian); infinite signatures contribute the identity
__global__ void __launch_bounds__(WG) k_mv_g2mul(const g2a *sigs, const uint64_t *rands, uint32_t n,
                                                 g2j *R) {
  uint32_t i = gtid();
  if (i >= n) return;
  g2j t;
  mul_u64(t, sigs[i], rands ? rands[i] : 1);
  R[i] = t;
}

// S_s = sum R_i over segment s; writes the segment's extra Miller pair (-g1, S_s)
// at index n + s of the pair arrays.
__global__ void __launch_bounds__(WGR) k_seg_g2_sum(const g2j *R, const uint32_t *off,
                                                    uint32_t nseg, uint32_t n, g1p *P, g2h *H) {
  uint32_t s = blockIdx.x;
  if (s >= nseg) return;
  g2j acc;
  jac_set_inf(acc);
  for (uint32_t i = off[s] + threadIdx.x; i < off[s + 1]; i += WGR) {
    g2j r = R[i];
    jac_add(acc, acc, r);
  }
  wg_reduce_jac(acc);
  if (threadIdx.x == 0) {
    g1a ng1;
    neg_g1_gen(ng1);
    g1p pp;
    g1p_from_aff(pp, ng1);
    g2h q;
    g2h_from_jac(q, acc);
    P[n + s] = pp;
    H[n + s] = q;
  }
}

// f_i = MillerLoop(P_i, H_i) over all pairs (sets and per-segment extra pairs)
__global__ void __launch_bounds__(WG) k_miller(const g1p *P, const g2h *H, uint32_t npairs,
                                               fp12 *f) {
  uint32_t i = gtid();
  if (i >= npairs) return;
  fp12 r;
  miller_loop(r, P[i], H[i]);
  f[i] = r;
}

// partial_s = f[n+s] * prod f_i over segment s;  err_s = OR bad_i | empty segment
__global__ void __launch_bounds__(WGR) k_seg_fp12_prod(const fp12 *f, const int32_t *bad,
                                                       const uint32_t *off, uint32_t nseg,
                                                       uint32_t n, fp12 *part, int32_t *err) {
  __shared__ fp12 buf[WGR / 2];
  __shared__ int32_t e_sh;
  uint32_t s = blockIdx.x;
  if (s >= nseg) return;
  if (threadIdx.x == 0) e_sh = 0;
  __syncthreads();
  fp12 acc;
  if (threadIdx.x == 0)
    acc = f[n + s];
  else
    fp12_one(acc);
  int32_t e = 0;
  for (uint32_t i = off[s] + threadIdx.x; i < off[s + 1]; i += WGR) {
    fp12 x = f[i];
    fp12_mul(acc, acc, x);
    e |= bad[i];
  }
  if (e) atomicOr(&e_sh, 1);
  for (int w = WGR / 2; w > 0; w >>= 1) {
    __syncthreads();
    if (threadIdx.x >= (unsigned)w && threadIdx.x < (unsigned)2 * w) buf[threadIdx.x - w] = acc;
    __syncthreads();
    if (threadIdx.x < (unsigned)w) {
      fp12 o = buf[threadIdx.x];
      fp12_mul(acc, acc, o);
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    part[s] = acc;
    err[s] = e_sh | (off[s + 1] == off[s] ? 1 : 0);
  }
}

// ---------------------------------------------------------------- final exponentiation
// product of nparts partials per segment (multi-GPU all-gather layout [part][seg]) and
// the easy part.
__global__ void __launch_bounds__(WG) k_fe_easy(const fp12 *part, const int32_t *err,
                                                uint32_t nparts, uint32_t nseg, fp12 *F,
                                                int32_t *err_out) {
  uint32_t s = gtid();
  if (s >= nseg) return;
  fp12 acc = part[s];
  int32_t e = err[s];
  for (uint32_t k = 1; k < nparts; k++) {
    fp12 o = part[(size_t)k * nseg + s];
    fp12_mul(acc, acc, o);
    e |= err[(size_t)k * nseg + s];
  }
  fp12 r;
  fe_easy(r, acc);
  F[s] = r;
  err_out[s] = e;
}
__global__ void __launch_bounds__(WG) k_fe_xm1(const fp12 *in, uint32_t nseg, fp12 *out) {
  uint32_t s = gtid();
  if (s >= nseg) return;
  fp12 a = in[s], r;
  fe_s_xm1(r, a);
  out[s] = r;
}
__global__ void __launch_bounds__(WG) k_fe_xpp(const fp12 *in, uint32_t nseg, fp12 *out) {
  uint32_t s = gtid();
  if (s >= nseg) return;
  fp12 a = in[s], r;
  fe_s_xpp(r, a);
  out[s] = r;
}
__global__ void __launch_bounds__(WG) k_fe_x(const fp12 *in, uint32_t nseg, fp12 *out) {
  uint32_t s = gtid();
  if (s >= nseg) return;
  fp12 a = in[s], r;
  fp12_cyc_exp_x(r, a);
  out[s] = r;
}
__global__ void __launch_bounds__(WG) k_fe_s5(const fp12 *T, const fp12 *B, uint32_t nseg,
                                              fp12 *out) {
  uint32_t s = gtid();
  if (s >= nseg) return;
  fp12 t = T[s], b = B[s], r;
  fe_s5(r, t, b);
  out[s] = r;
}
__global__ void __launch_bounds__(WG) k_fe_s6(const fp12 *C, const fp12 *F, const int32_t *err,
                                              uint32_t nseg, int32_t *verdict) {
  uint32_t s = gtid();
  if (s >= nseg) return;
  fp12 c = C[s], f = F[s], r;
  fe_s6(r, c, f);
  verdict[s] = (!err[s] && fp12_is_one(r)) ? ST_SUCCESS : ST_VERIFY_FAIL;
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

}  // namespace gbls
