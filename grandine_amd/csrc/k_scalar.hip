// gfx950 kernels: the random linear combination of Signature::multi_verify
// (bls/src/signature.rs:106-126): P_i = r_i pk_i (G1, one lane per set) and
// S = sum r_i sig_i (G2, one lane per set + a workgroup tree per segment).
#include "gbls_common.h"

namespace gbls {

// P_i = affine(r_i pk_i); bad_i = pk infinite (blst PAIRING_Aggregate_PK_in_G1 rejects
// it) or a caller pre-check failed (signature subgroup check, aggregation status).
__global__ void __launch_bounds__(WG) k_mv_g1mul(const g1a *pks, const uint64_t *rands,
                                                 const int32_t *pre, uint32_t n, g1a *P,
                                                 int32_t *bad) {
  uint32_t i = blockIdx.x * WG + threadIdx.x;
  if (i >= n) return;
  g1a pk = pks[i];
  uint64_t r = rands ? rands[i] : 1;
  g1j t;
  mul_u64(t, pk, r);
  g1a o;
  jac_to_aff(o, t);
  P[i] = o;
  bad[i] = (aff_is_inf(pk) || (pre && pre[i] != 0)) ? 1 : 0;
}

// R_i = r_i sig_i (Jacobian); infinite signatures contribute the identity (blst skips
// them in the G2 accumulation)
__global__ void __launch_bounds__(WG) k_mv_g2mul(const g2a *sigs, const uint64_t *rands, uint32_t n,
                                                 g2j *R) {
  uint32_t i = blockIdx.x * WG + threadIdx.x;
  if (i >= n) return;
  g2j t;
  mul_u64(t, sigs[i], rands ? rands[i] : 1);
  R[i] = t;
}

template <class F>
__device__ void wg_reduce_jac2(jac<F> &v) {
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

// S_s = sum R_i over segment s -> the segment's extra Miller pair (-g1, S_s) at index
// n + s of the pair arrays; seg_err[s] = OR bad_i | (segment empty)
__global__ void __launch_bounds__(WGR) k_seg_g2_sum(const g2j *R, const int32_t *bad,
                                                    const uint32_t *off, uint32_t nseg, uint32_t n,
                                                    g1a *P, g2a *H, int32_t *seg_err) {
  __shared__ int32_t e_sh;
  uint32_t s = blockIdx.x;
  if (s >= nseg) return;
  if (threadIdx.x == 0) e_sh = 0;
  __syncthreads();
  g2j acc;
  jac_set_inf(acc);
  int32_t e = 0;
  for (uint32_t i = off[s] + threadIdx.x; i < off[s + 1]; i += WGR) {
    g2j r = R[i];
    jac_add(acc, acc, r);
    e |= bad[i];
  }
  if (e) atomicOr(&e_sh, 1);
  wg_reduce_jac2(acc);
  if (threadIdx.x == 0) {
    g1a ng1;
    fp_set(ng1.x, k::G1X_M);
    fp_set(ng1.y, k::G1NEGY_M);
    g2a q;
    jac_to_aff(q, acc);
    P[n + s] = ng1;
    H[n + s] = q;
    seg_err[s] = e_sh | (off[s + 1] == off[s] ? 1 : 0);
  }
}

void launch_mv_g1mul(hipStream_t st, const g1a *pks, const uint64_t *rands, const int32_t *pre,
                     uint32_t n, g1a *P, int32_t *bad) {
  k_mv_g1mul<<<nblk(n), WG, 0, st>>>(pks, rands, pre, n, P, bad);
}
void launch_mv_g2mul(hipStream_t st, const g2a *sigs, const uint64_t *rands, uint32_t n, g2j *R) {
  k_mv_g2mul<<<nblk(n), WG, 0, st>>>(sigs, rands, n, R);
}
void launch_seg_g2_sum(hipStream_t st, const g2j *R, const int32_t *bad, const uint32_t *seg_off,
                       uint32_t nseg, uint32_t n, g1a *P, g2a *H, int32_t *seg_err) {
  k_seg_g2_sum<<<nseg, WGR, 0, st>>>(R, bad, seg_off, nseg, n, P, H, seg_err);
}

}  // namespace gbls
