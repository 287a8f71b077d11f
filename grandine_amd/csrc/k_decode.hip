// gfx950 kernels: point encodings (a8, a9, a10) and the signature subgroup check,
// one lane per point.

#include "gbls_common.h"
#include "bls_w4.h"
#include "bls_curve28.h"

namespace gbls {

__global__ void __launch_bounds__(WG) k_g1_decompress(const uint8_t *in, uint32_t n, int validate,
                                                      g1a *out, int32_t *st) {
  uint32_t i = blockIdx.x * WG + threadIdx.x;
  if (i >= n) return;
  g1a a;
  int32_t s = g1_decompress(a, in + 48u * i);
  if (s == ST_SUCCESS && validate) {  // PublicKey::validate, public_key.rs:27
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

template <bool X>
__global__ void __launch_bounds__(WG) k_g2_decompress(const uint8_t *in, uint32_t n, g2a *out,
                                                      int32_t *st) {
  if constexpr (X) w4::exclusive_simd();
  uint32_t i = blockIdx.x * WG + threadIdx.x;
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

// one 16-lane row per signature (the latency regime: blocks' MultiVerifier::finish): the two
// (p-3)/4 exponentiations of the Fp2 square root row-distributed (bls_dfp.h), ~2.5x faster
// per product than one lane's; the rest of the decoding runs redundantly on the row's lanes
struct RowPowDec {
  __device__ void operator()(fp &r, const fp &a) const {
    dfp::Tabs t;
    dfp::load_tabs(t);
    const uint32_t x = dfp::pow_pm3d4(dfp::from_regs(a.l, t), t);
    dfp::to_words_all(r.l, x, t);
  }
};
template <bool X>
__global__ void __launch_bounds__(WG) k_g2_decompress_row(const uint8_t *in, uint32_t n, g2a *out,
                                                          int32_t *st) {
  if constexpr (X) w4::exclusive_simd();
  const uint32_t i = (blockIdx.x * WG + threadIdx.x) >> 4;
  if (i >= n) return;  // whole rows
  g2a a;
  int32_t s = g2_decompress_pow(a, in + 96u * i, RowPowDec());
  if (s != ST_SUCCESS) {
    fp2_zero(a.x);
    fp2_zero(a.y);
  }
  if ((threadIdx.x & 15) == 0) {
    out[i] = a;
    st[i] = s;
  }
}
constexpr uint32_t kDecRowsMax = 2048;  // signatures up to this many take the row form

// signature subgroup check (sig_groupcheck = true in verify / fast_aggregate_verify,
// signature.rs:51,86); infinity passes.  st[i] |= 1 on failure when `accumulate`.
__global__ void __launch_bounds__(WG) k_g2_check(const g2a *in, uint32_t n, int32_t *st,
                                                 int accumulate) {
  uint32_t i = blockIdx.x * WG + threadIdx.x;
  if (i >= n) return;
  g2a a = in[i];
  bool ok = aff_is_inf(a) || (g2_on_curve(a) && g2_in_group(a));
  if (accumulate)
    st[i] = st[i] | (ok ? 0 : 1);
  else
    st[i] = ok ? ST_SUCCESS : ST_NOT_IN_GROUP;
}

// the same with the membership chain in radix 2^28 (bls_curve28.h g2_in_group28: lazy
// doublings, mixed additions of the base, which waits in LDS at an odd stride of 57 words)
__global__ void __launch_bounds__(WG) k_g2_check28(const g2a *in, uint32_t n, int32_t *st,
                                                   int accumulate) {
  uint32_t i = blockIdx.x * WG + threadIdx.x;
  if (i >= n) return;
  struct g2a28_lds {
    r28::g2a28 v;
    uint32_t pad;
  };
  static_assert(sizeof(g2a28_lds) == 57 * 4, "odd LDS stride");
  __shared__ g2a28_lds bl[WG];
  const g2a a = in[i];
  bool ok = aff_is_inf(a);
  if (!ok && g2_on_curve(a)) {
    r28::g2a28 &b = bl[threadIdx.x].v;
    r28::g2a28 t;
    r28::from_fp(t.x.c0, a.x.c0), r28::from_fp(t.x.c1, a.x.c1);
    r28::from_fp(t.y.c0, a.y.c0), r28::from_fp(t.y.c1, a.y.c1);
    b = t;
    ok = r28::g2_in_group28(b);
  }
  if (accumulate)
    st[i] = st[i] | (ok ? 0 : 1);
  else
    st[i] = ok ? ST_SUCCESS : ST_NOT_IN_GROUP;
}

__global__ void __launch_bounds__(WG) k_g1_compress(const g1a *in, uint32_t n, uint8_t *out) {
  uint32_t i = blockIdx.x * WG + threadIdx.x;
  if (i >= n) return;
  g1_compress(out + 48u * i, in[i]);
}
__global__ void __launch_bounds__(WG) k_g2_compress(const g2a *in, uint32_t n, uint8_t *out) {
  uint32_t i = blockIdx.x * WG + threadIdx.x;
  if (i >= n) return;
  g2_compress(out + 96u * i, in[i]);
}

// ---------------------------------------------------------------- launchers
void launch_g1_decompress(hipStream_t st, const uint8_t *in, uint32_t n, int validate, g1a *out,
                          int32_t *status) {
  if (n) k_g1_decompress<<<nblk(n), WG, 0, st>>>(in, n, validate, out, status);
}
void launch_g2_decompress(hipStream_t st, const uint8_t *in, uint32_t n, g2a *out, int32_t *status) {
  if (n && n <= kDecRowsMax)
    (nblk(16 * (size_t)n) <= w4::kExclusiveMaxWaves ? k_g2_decompress_row<true> : k_g2_decompress_row<false>)<<<
        nblk(16 * (size_t)n), WG, 0, st>>>(in, n, out, status);
  else if (n)
    (nblk(n) <= w4::kExclusiveMaxWaves ? k_g2_decompress<true> : k_g2_decompress<false>)<<<nblk(n), WG, 0, st>>>(
        in, n, out, status);
}
void launch_g2_check(hipStream_t st, const g2a *in, uint32_t n, int32_t *status, int accumulate) {
  if (!n) return;
  if (g_lane_r28)
    k_g2_check28<<<nblk(n), WG, 0, st>>>(in, n, status, accumulate);
  else
    k_g2_check<<<nblk(n), WG, 0, st>>>(in, n, status, accumulate);
}
void launch_g1_compress(hipStream_t st, const g1a *in, uint32_t n, uint8_t *out) {
  if (n) k_g1_compress<<<nblk(n), WG, 0, st>>>(in, n, out);
}
void launch_g2_compress(hipStream_t st, const g2a *in, uint32_t n, uint8_t *out) {
  if (n) k_g2_compress<<<nblk(n), WG, 0, st>>>(in, n, out);
}

}  // namespace gbls
