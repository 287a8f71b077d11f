// gfx950 kernels: hash_to_G2 (a13, RFC 9380 BLS12381G2_XMD:SHA-256_SSWU_RO_ with the
// Ethereum POP DST, bls/src/consts.rs:1) stage 3 (Q0 + Q1, cofactor clearing, affine).
// One DPP quad (4 lanes) per message: the doublings and additions run quad-cooperatively
// (bls_gang.h); psi and the affine conversion run
// redundantly in all four lanes and lane 0 stores.  Output: affine points (Miller-loop
// input).  Launches of at least g_lane_min messages run one message per lane in two
// kernels, one [|x|] chain each (k_h2c_clear_lane_a / _b, radix-2^28 by default: a quarter of
// the instructions per message, the chip already full).
#include "gbls_common.h"
#include "bls_gang.h"
#include "bls_w4.h"
#include "bls_curve28.h"

namespace gbls {

// Same sequence as clear_cofactor_g2 (bls_hash.h), with quad doublings and additions.
__device__ __forceinline__ void gang_clear_cofactor_g2(g2j &r, const g2j &p, int q) {
  g2j t1, t2, t3;
  gang_mul_by_xabs(t1, p, q);
  jac_neg(t1, t1);        // t1 = [x]P
  g2_psi(t2, p);
  gang_add(t2, t2, t1, q);    // t1 + psi(P)
  gang_mul_by_xabs(t3, t2, q);
  jac_neg(t3, t3);        // t3 = [x](t1 + psi(P))
  jac_neg(t1, t1);
  gang_add(t3, t3, t1, q);    // - t1
  gang_dbl(t1, p, q);
  g2_psi2(t1, t1);
  gang_add(t3, t3, t1, q);    // + psi^2(2P)
  g2_psi(t1, p);
  jac_neg(t1, t1);
  gang_add(t3, t3, t1, q);    // - psi(P)
  jac_neg(t1, p);
  gang_add(r, t3, t1, q);     // - P
}

// stage 3: Q0 + Q1, clear the cofactor (Budroni-Pintore), affine.  4 lanes per message;
// a quad never straddles the n boundary (the whole quad returns together).
// P = Q0 + Q1 waits in LDS (72 words per lane) while the chains run: 35 spilled VGPRs (48 B of
// scratch per lane) down to 3 (12 B, ten scratch instructions in the kernel)
__global__ void __launch_bounds__(WG) k_h2c_clear(const g2j *Q, uint32_t n, g2a *H) {
  uint32_t t = blockIdx.x * WG + threadIdx.x;
  uint32_t i = t >> 2;
  int q = (int)(t & 3);
  if (i >= n) return;
  __shared__ g2j pl[WG];
  g2j h;
  {
    g2j a = Q[2 * i], b = Q[2 * i + 1];
    gang_add(a, a, b, q);
    pl[threadIdx.x] = a;
  }
  gang_clear_cofactor_g2(h, pl[threadIdx.x], q);
  g2a o;
  jac_to_aff(o, h);
  if (q == 0) H[i] = o;
}

// Same sequence on a 16-lane row (tiny launches: the latency regime)
__device__ __forceinline__ void row_clear_cofactor_g2(g2j &r, const g2j &p, int l) {
  g2j t1, t2, t3;
  row_mul_by_xabs(t1, p, l);
  jac_neg(t1, t1);        // t1 = [x]P
  g2_psi(t2, p);
  row_add(t2, t2, t1, l);     // t1 + psi(P)
  row_mul_by_xabs(t3, t2, l);
  jac_neg(t3, t3);        // t3 = [x](t1 + psi(P))
  jac_neg(t1, t1);
  row_add(t3, t3, t1, l);     // - t1
  row_dbl(t1, p, l);
  g2_psi2(t1, t1);
  row_add(t3, t3, t1, l);     // + psi^2(2P)
  g2_psi(t1, p);
  jac_neg(t1, t1);
  row_add(t3, t3, t1, l);     // - psi(P)
  jac_neg(t1, p);
  row_add(r, t3, t1, l);      // - P
}
__global__ void __launch_bounds__(WG) k_h2c_clear_row(const g2j *Q, uint32_t n, g2a *H) {
  uint32_t t = blockIdx.x * WG + threadIdx.x;
  uint32_t i = t >> 4;
  int l = (int)(t & 15);
  if (i >= n) return;  // whole rows
  g2j a = Q[2 * i], b = Q[2 * i + 1], h;
  row_add(a, a, b, l);
  row_clear_cofactor_g2(h, a, l);
  g2a o;
  jac_to_aff(o, h);
  if (l == 0) H[i] = o;
}

// The lane form in two kernels, one [|x|] chain each: in one kernel P and
// t1 = [x]P stay live through the second chain next to its base and accumulator, and the
// kernel spilled 100 B per lane; here each chain holds only its base, its accumulator and the
// addition's temporaries, and the points between the chains wait in the message's own two Q
// slots in HBM (576 B per message).  The same group element as clear_cofactor_g2 (RFC 9380
// G.3 order):
//   a: P = Q0 + Q1;  t1 = [x]P;  t2 = t1 + psi(P) -> Q[2i];  T = psi^2(2P) - psi(P) - P - t1 -> Q[2i+1]
//   b: h = [x] t2 + T -> affine H[i]
__global__ void __launch_bounds__(WG) k_h2c_clear_lane_a(g2j *Q, uint32_t n) {
  const uint32_t i = blockIdx.x * WG + threadIdx.x;
  if (i >= n) return;
  g2j p = Q[2 * i], t1;
  {
    const g2j q1 = Q[2 * i + 1];
    jac_add(p, p, q1);
  }
  mul_by_xabs(t1, p);
  jac_neg(t1, t1);  // t1 = [x]P
  {
    g2j t2;
    g2_psi(t2, p);
    jac_add(t2, t2, t1);  // t2 = t1 + psi(P)
    Q[2 * i] = t2;
  }
  jac_neg(t1, t1);  // -t1
  {
    g2j v;
    jac_neg(v, p);
    jac_add(t1, t1, v);  // - t1 - P
    jac_dbl(v, p);
    g2_psi2(v, v);
    jac_add(t1, t1, v);  // + psi^2(2P)
    g2_psi(v, p);
    jac_neg(v, v);
    jac_add(t1, t1, v);  // - psi(P)
  }
  Q[2 * i + 1] = t1;
}
__global__ void __launch_bounds__(WG) k_h2c_clear_lane_b(const g2j *Q, uint32_t n, g2a *H) {
  const uint32_t i = blockIdx.x * WG + threadIdx.x;
  if (i >= n) return;
  g2j h;
  {
    const g2j t2 = Q[2 * i];
    mul_by_xabs(h, t2);
  }
  jac_neg(h, h);  // [x] t2
  {
    const g2j T = Q[2 * i + 1];
    jac_add(h, h, T);
  }
  g2a o;
  jac_to_aff(o, h);
  H[i] = o;
}

// The two lane-form chains in radix 2^28 (bls_curve28.h: the engine's Jacobian templates over
// r28::fe2, one v_mad_u64_u32 per product term), the default since r05 (g_lane_r28).  The chain's
// base point waits in LDS for its 5 additions (84 words per lane), which keeps both kernels
// free of scratch; between the chains the message's Q slots hold the radix-2^28 limbs repacked
// into the engine layout (store12, no conversion product); chain b converts its result to
// engine form (to_fp) before the affine conversion, so H is bit-identical to the 32-bit path's.
__device__ __forceinline__ void g2j28_store(g2j &dst, const r28::g2j28 &a) { r28::g2j_store12(dst, a); }
__device__ __forceinline__ void g2j28_load(r28::g2j28 &r, const g2j &src) { r28::g2j_load12(r, src); }
// A chain's base point in LDS, one per lane at an ODD stride of 85 words (84 + 1 pad): the 4-byte
// LDS accesses of the 32 lanes of a group then fall in 32 different banks (the unpadded stride
// of 84 = 4 x 21 words put every 4th lane on one bank: 4-way conflicts, 58 % of the kernels'
// LDS cycles in the r05 PMC pass, SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE)
struct g2j28_lds {
  r28::g2j28 v;
  uint32_t pad;
};
static_assert(sizeof(g2j28_lds) == 85 * 4, "odd LDS stride");
// h = [|x|] (*pl), the base read from LDS at each of the 5 additions
__device__ __forceinline__ void mul_by_xabs28(r28::g2j28 &h, const r28::g2j28 *pl) {
  h = *pl;
  for (int b = 62; b >= 0; b--) {
    jac_dbl(h, h);
    if ((k::X_ABS >> b) & 1) jac_add(h, h, *pl);
  }
}
__global__ void __launch_bounds__(WG) k_h2c_clear_lane_a28(g2j *Q, uint32_t n) {
  const uint32_t i = blockIdx.x * WG + threadIdx.x;
  if (i >= n) return;
  __shared__ g2j28_lds pl[WG];
  r28::g2j28 *pp = &pl[threadIdx.x].v;
  r28::g2j28 t1;
  {
    r28::g2j28 p, q;
    const g2j e0 = Q[2 * i];
    r28::g2j_in(p, e0);
    const g2j e1 = Q[2 * i + 1];
    r28::g2j_in(q, e1);
    jac_add(p, p, q);  // P = Q0 + Q1
    *pp = p;
  }
  mul_by_xabs28(t1, pp);
  jac_neg(t1, t1);  // t1 = [x]P
  {
    r28::g2j28 t2;
    r28::g2_psi28(t2, *pp);
    jac_add(t2, t2, t1);  // t2 = t1 + psi(P)
    g2j28_store(Q[2 * i], t2);
  }
  jac_neg(t1, t1);  // -t1
  {
    r28::g2j28 v;
    jac_neg(v, *pp);
    jac_add(t1, t1, v);  // - t1 - P
    jac_dbl(v, *pp);
    r28::g2_psi2_28(v, v);
    jac_add(t1, t1, v);  // + psi^2(2P)
    r28::g2_psi28(v, *pp);
    jac_neg(v, v);
    jac_add(t1, t1, v);  // - psi(P)
  }
  g2j28_store(Q[2 * i + 1], t1);
}
__global__ void __launch_bounds__(WG) k_h2c_clear_lane_b28(const g2j *Q, uint32_t n, g2a *H) {
  const uint32_t i = blockIdx.x * WG + threadIdx.x;
  if (i >= n) return;
  __shared__ g2j28_lds pl[WG];
  r28::g2j28 *pp = &pl[threadIdx.x].v;
  r28::g2j28 h;
  {
    r28::g2j28 t2;
    g2j28_load(t2, Q[2 * i]);
    *pp = t2;
  }
  mul_by_xabs28(h, pp);
  jac_neg(h, h);  // [x] t2
  {
    r28::g2j28 T;
    g2j28_load(T, Q[2 * i + 1]);
    *pp = T;
    jac_add(h, h, *pp);
  }
  g2j e;
  r28::g2j_out(e, h);
  g2a o;
  jac_to_aff(o, e);
  H[i] = o;
}

// The staged form (GBLS_CLEAR_STAGED=1, off by default; bls_curve28.h clear_mid28): both
// [|x|] chains run on AFFINE bases in their own kernel, k_h2c_chain28, whose 63 lazy doublings
// and 5 mixed additions fit 256 VGPRs without scratch: two waves per SIMD, so a chain launch
// shares its SIMDs with the other in-flight submission's waves (the one-kernel chains above take
// 256 VGPRs + ~250 AGPRs for the Jacobian base's full additions).  The affine conversions cost
// one safegcd inversion each (pre, mid).  Per message the Q slots carry, in radix-2^28 limbs:
//   pre:   Q[2i] = P = Q0 + Q1 (affine x, y)
//   chain: Q[2i+1] = X1 = [|x|] P
//   mid:   Q[2i] = t2 = [x]P + psi(P) (affine), Q[2i+1] = T = X1 - P + psi^2(2P) - psi(P)
//   chain: Q[2i] = X2 = [|x|] t2
//   post:  H[i] = affine(T - X2), engine form
// Measured (profiles/r06/y_ab_clear_staged.txt, one box): C2 4.57-4.72M against 4.63-4.69M, C3
// 795-824k against 827-855k.  A chain launch of one submission is 1024 waves, one per SIMD, and
// the other submission's kernels take 512 registers per wave, so the second wave slot is rarely
// used, while the affine conversions and the extra launches cost.  Kept as a knob.
__device__ __forceinline__ g2a &q_aff(g2j &slot) { return *reinterpret_cast<g2a *>(&slot); }
__global__ void __launch_bounds__(WG) k_h2c_clear_pre28(g2j *Q, uint32_t n) {
  const uint32_t i = blockIdx.x * WG + threadIdx.x;
  if (i >= n) return;
  r28::g2j28 p, q;
  r28::g2j_in(p, Q[2 * i]);
  r28::g2j_in(q, Q[2 * i + 1]);
  jac_add(p, p, q);
  r28::g2a28 a;
  r28::jac_to_aff28(a, p);
  r28::g2a_store12(q_aff(Q[2 * i]), a);
}
struct g2a28_lds {
  r28::g2a28 v;
  uint32_t pad;
};
static_assert(sizeof(g2a28_lds) == 57 * 4, "odd LDS stride");
template <int SRC, int DST>
__global__ void __launch_bounds__(WG) __attribute__((amdgpu_waves_per_eu(2, 2)))
k_h2c_chain28(g2j *Q, uint32_t n) {
  const uint32_t i = blockIdx.x * WG + threadIdx.x;
  if (i >= n) return;
  __shared__ g2a28_lds bl[WG];
  r28::g2a28 &b = bl[threadIdx.x].v;
  {
    r28::g2a28 t;
    r28::g2a_load12(t, q_aff(Q[2 * i + SRC]));
    b = t;
  }
  r28::g2j28 h;
  r28::g2_xabs_aff28(h, b);
  r28::g2j_store12(Q[2 * i + DST], h);
}
__global__ void __launch_bounds__(WG) k_h2c_clear_mid28(g2j *Q, uint32_t n) {
  const uint32_t i = blockIdx.x * WG + threadIdx.x;
  if (i >= n) return;
  r28::g2a28 pa, t2a;
  r28::g2j28 x1, T;
  r28::g2a_load12(pa, q_aff(Q[2 * i]));
  r28::g2j_load12(x1, Q[2 * i + 1]);
  r28::clear_mid28(t2a, T, pa, x1);
  r28::g2a_store12(q_aff(Q[2 * i]), t2a);
  r28::g2j_store12(Q[2 * i + 1], T);
}
__global__ void __launch_bounds__(WG) k_h2c_clear_post28(const g2j *Q, uint32_t n, g2a *H) {
  const uint32_t i = blockIdx.x * WG + threadIdx.x;
  if (i >= n) return;
  r28::g2j28 x2, T, h;
  r28::g2j_load12(x2, Q[2 * i]);
  r28::g2j_load12(T, Q[2 * i + 1]);
  r28::clear_post28(h, x2, T);
  g2j e;
  r28::g2j_out(e, h);
  g2a o;
  jac_to_aff(o, e);
  H[i] = o;
}

// one wave per message (bls_w4.h: four row-distributed products per round), the smallest
// launches: Q0 + Q1, the cofactor clearing and the affine conversion at ~0.5 us per round
template <bool X>
__global__ void __launch_bounds__(64) k_h2c_clear_w4(const g2j *Q, uint32_t n, g2a *H) {
  if constexpr (X) w4::exclusive_simd();
  const uint32_t i = blockIdx.x;
  if (i >= n) return;  // whole waves
  w4::Ctx c;
  w4::init(c);
  w4::J a, b, h;
  w4::load(c, a, Q[2 * i]);
  w4::load(c, b, Q[2 * i + 1]);
  w4::add(c, a, a, b);
  w4::clear_cofactor(c, h, a);
  w4::store_affine(c, H + i, h);
}

// the pipeline's form: the cleared point stays Jacobian (no inversion: the Miller lines take
// it projectively), written over Q[2 i]
template <bool X>
__global__ void __launch_bounds__(64) k_h2c_clear_w4j(g2j *Q, uint32_t n) {
  if constexpr (X) w4::exclusive_simd();
  const uint32_t i = blockIdx.x;
  if (i >= n) return;  // whole waves
  w4::Ctx c;
  w4::init(c);
  w4::J a, b, h;
  w4::load(c, a, Q[2 * i]);
  w4::load(c, b, Q[2 * i + 1]);
  w4::add(c, a, a, b);
  w4::clear_cofactor(c, h, a);
  w4::store_jac(c, Q + 2 * i, h);
}
bool launch_h2c_clear_jac(hipStream_t st, g2j *Q, uint32_t n) {
  if (!n || n > kW4Max) return false;
  (n <= w4::kExclusiveMaxWaves ? k_h2c_clear_w4j<true> : k_h2c_clear_w4j<false>)<<<n, 64, 0, st>>>(Q, n);
  return true;
}

void launch_h2c_clear(hipStream_t st, const g2j *Q, uint32_t n, g2a *H) {
  if (!n) return;
  if (n <= kW4Max)
    (n <= w4::kExclusiveMaxWaves ? k_h2c_clear_w4<true> : k_h2c_clear_w4<false>)<<<n, 64, 0, st>>>(Q, n, H);
  else if (n >= g_lane_min) {
    // Q is a scratch of the call (the map's output); its two slots per message carry the
    // points between the two chains
    g2j *Qw = const_cast<g2j *>(Q);
    if (g_lane_r28 && g_clear_staged) {
      k_h2c_clear_pre28<<<nblk(n), WG, 0, st>>>(Qw, n);
      k_h2c_chain28<0, 1><<<nblk(n), WG, 0, st>>>(Qw, n);
      k_h2c_clear_mid28<<<nblk(n), WG, 0, st>>>(Qw, n);
      k_h2c_chain28<0, 0><<<nblk(n), WG, 0, st>>>(Qw, n);
      k_h2c_clear_post28<<<nblk(n), WG, 0, st>>>(Q, n, H);
    } else if (g_lane_r28) {
      k_h2c_clear_lane_a28<<<nblk(n), WG, 0, st>>>(Qw, n);
      k_h2c_clear_lane_b28<<<nblk(n), WG, 0, st>>>(Q, n, H);
    } else {
      k_h2c_clear_lane_a<<<nblk(n), WG, 0, st>>>(const_cast<g2j *>(Q), n);
      k_h2c_clear_lane_b<<<nblk(n), WG, 0, st>>>(Q, n, H);
    }
  }
  else if (n <= g_row_clear_max)
    k_h2c_clear_row<<<nblk((size_t)n * 16), WG, 0, st>>>(Q, n, H);
  else
    k_h2c_clear<<<nblk((size_t)n * 4), WG, 0, st>>>(Q, n, H);
}

}  // namespace gbls
