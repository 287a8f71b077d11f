// gfx950 kernels: the batch Miller product as a tree (bls_pairing.h header comment).
//   k_ml_group  lane per (event e, group of <= G pairs of one segment): the product of
//               the group's evaluated lines, line_e(P_a) line_e(P_b) ... (sparse x sparse,
//               then dense x sparse), in registers -> one dense Fp12.  A group's pairs are
//               strided through its segment's pair list (pair k, k + ng, k + 2 ng, ...
//               for ng groups), so lanes of a wave load the SoA line words of adjacent
//               pairs: coalesced.  G grows with the batch (bigger G = fewer values for
//               the wave-cooperative levels, which are 3x less efficient per product).
//   k_ml_reduce wave per (event, group of <= 4 values of one segment): wave-cooperative
//               Fp12 products (bls_wave12.h)
//   k_ml_horner wave per segment: Horner over the 68 events, then conj (x < 0)
#include "bls_wave12.h"
#include "bls_w12d.h"
#include "bls_field28.h"
#include "gbls_common.h"

namespace gbls {

__device__ __forceinline__ void ml_eval(sp034 &s, const uint32_t *L, uint32_t np, const g1s *P,
                                        uint32_t pair, int e) {
  fp2 L0, L2, L3;
  line_get(L, np, pair, e, L0, L2, L3);
  g1s Pp = P[pair];
  line_eval_s(s, L0, L2, L3, Pp);
}

// grid (ceil(ngroup / 64), e1 - e0); group g = (first plist index, stride, count); the
// lines buffer holds events [e0, e1) at e - e0
__global__ void __launch_bounds__(WG) k_ml_group(const uint32_t *L, uint32_t np, const g1s *P,
                                                 const uint32_t *plist, const uint32_t *grp,
                                                 uint32_t ngroup, int e0, fp12 *V0) {
  uint32_t g = blockIdx.x * WG + threadIdx.x;
  int el = blockIdx.y, e = e0 + el;
  if (g >= ngroup) return;
  uint32_t at = grp[3 * g], stride = grp[3 * g + 1], cnt = grp[3 * g + 2];
  sp034 sa, sb;
  fp12 acc;
  ml_eval(sa, L, np, P, plist[at], el);
  if (cnt == 1) {
    sp_to_fp12(acc, sa);
  } else {
    ml_eval(sb, L, np, P, plist[at + stride], el);
    sp_mul_sp(acc, sa, sb);
    for (uint32_t j = 2; j < cnt; j++) {
      ml_eval(sa, L, np, P, plist[at + j * stride], el);
      fp12_mul_034(acc, acc, sa);
    }
  }
  V0[(size_t)e * ngroup + g] = acc;
}

#ifdef GBLS_EXPERIMENTS  // measured slower; not in the shipped build
// k_ml_group in radix-2^28 arithmetic (bls_field28.h; GBLS_ML_R28=1): same grid, same
// inputs, and an output that differs from k_ml_group's by an Fp scalar (2^-16 per line and
// 2^8 from the engine-form reading), which the final exponentiation removes
__device__ __forceinline__ void ml_eval28(r28::sp &s, const uint32_t *L, uint32_t np, const g1s *P,
                                          uint32_t pair, int e) {
  fp2 L0, L2, L3;
  line_get(L, np, pair, e, L0, L2, L3);
  const g1s &Pp = P[pair];
  if (fp_is_zero(Pp.c))
    r28::sp_identity(s);
  else
    r28::sp_from_engine(s, L0, L2, L3, Pp.x, Pp.y, Pp.c);
}
__global__ void __launch_bounds__(WG) k_ml_group28(const uint32_t *L, uint32_t np, const g1s *P,
                                                   const uint32_t *plist, const uint32_t *grp,
                                                   uint32_t ngroup, int e0, fp12 *V0) {
  uint32_t g = blockIdx.x * WG + threadIdx.x;
  int el = blockIdx.y, e = e0 + el;
  if (g >= ngroup) return;
  uint32_t at = grp[3 * g], stride = grp[3 * g + 1], cnt = grp[3 * g + 2];
  __shared__ uint32_t stash[154 * WG];
  r28::sp sa, sb;
  r28::fe12 acc;
  ml_eval28(sa, L, np, P, plist[at], el);
  if (cnt == 1) {
    r28::sp_to_fe12(acc, sa);
  } else {
    ml_eval28(sb, L, np, P, plist[at + stride], el);
    r28::sp_mul_sp(acc, sa, sb);
    for (uint32_t j = 2; j < cnt; j++) {
      ml_eval28(sa, L, np, P, plist[at + j * stride], el);
      r28::fe12_mul_034_st(acc, acc, sa, stash + threadIdx.x, WG);
    }
  }
  fp12 out;
  r28::fe12_to_engine_scaled(out, acc);
  V0[(size_t)e * ngroup + g] = out;
}

#endif  // GBLS_EXPERIMENTS

// copy one Fp12 image global <-> LDS with all 64 lanes
__device__ __forceinline__ void w12_load(uint32_t *dst, const fp12 *src) {
  const uint32_t *s = reinterpret_cast<const uint32_t *>(src);
  for (int i = threadIdx.x; i < W12_WORDS; i += 64) dst[i] = s[i];
  __syncthreads();
}
__device__ __forceinline__ void w12_store(fp12 *dst, const uint32_t *src) {
  uint32_t *d = reinterpret_cast<uint32_t *>(dst);
  for (int i = threadIdx.x; i < W12_WORDS; i += 64) d[i] = src[i];
}

// grid (nout, 68): output q of event e = product of Vin[e][red[2q] .. red[2q]+red[2q+1])
__global__ void __launch_bounds__(64) k_ml_reduce(const fp12 *Vin, uint32_t nin, const uint32_t *red,
                                                  uint32_t nout, fp12 *Vout) {
  W12_SHARED uint32_t acc[W12_WORDS], tmp[W12_WORDS], ws[W12_WS_WORDS];
  w12_plan pl;
  w12_begin(pl, ws);
  uint32_t q = blockIdx.x;
  int e = blockIdx.y;
  uint32_t b = red[2 * q], cnt = red[2 * q + 1];
  const fp12 *src = Vin + (size_t)e * nin + b;
  w12_load(acc, src);
  for (uint32_t j = 1; j < cnt; j++) {
    w12_load(tmp, src + j);
    w12_mul(pl, acc, acc, tmp, ws);
  }
  w12_store(Vout + (size_t)e * nout + q, acc);
}

// grid nseg: V holds one value per (event, segment): V[e * nseg + s]
__global__ void __launch_bounds__(64) k_ml_horner(const fp12 *V, uint32_t nseg, fp12 *partial,
                                                  const uint32_t *lim, uint32_t base) {
  W12_SHARED uint32_t acc[W12_WORDS], tmp[W12_WORDS], ws[W12_WS_WORDS];
  uint32_t s = blockIdx.x;
  if (lim && base + s >= *lim) return;  // block-uniform
  w12_plan pl;
  w12_begin(pl, ws);
  w12_load(acc, V + s);
  for (int e = 1; e < ML_EVENTS; e++) {
    if (ev_is_dbl(e)) w12_mul(pl, acc, acc, acc, ws);
    w12_load(tmp, V + (size_t)e * nseg + s);
    w12_mul(pl, acc, acc, tmp, ws);
  }
  w12_conj(acc, acc);
  w12_store(partial + s, acc);
}

void launch_ml_group(hipStream_t st, const uint32_t *lines, uint32_t np, const g1s *P,
                     const uint32_t *plist, const uint32_t *groups, uint32_t ngroup, int e0,
                     int e1, fp12 *V0) {
  dim3 grid(nblk(ngroup), e1 - e0);
  if (!ngroup || e1 <= e0) return;
#ifdef GBLS_EXPERIMENTS
  if (g_ml_r28) {
    k_ml_group28<<<grid, WG, 0, st>>>(lines, np, P, plist, groups, ngroup, e0, V0);
    return;
  }
#endif
  k_ml_group<<<grid, WG, 0, st>>>(lines, np, P, plist, groups, ngroup, e0, V0);
}
void launch_ml_reduce(hipStream_t st, const fp12 *Vin, uint32_t nin, const uint32_t *red,
                      uint32_t nout, fp12 *Vout) {
  dim3 grid(nout, ML_EVENTS);
  if (nout) k_ml_reduce<<<grid, 64, 0, st>>>(Vin, nin, red, nout, Vout);
}
// k_ml_horner on the row-distributed Fp12 engine (bls_w12d.h), for launches of a few
// segments, with the 68-event chain SPLIT into parts that run side by side (one workgroup
// each, grid (nseg, parts)): f = prod_k V_k^(2^(D_k)) (D_k = doubling events after k), so part
// [a, b) computes its own Horner value and then squares it once per doubling event after b;
// the parts' products are f.  With 4 parts the longest chain is 53.5 product-times instead of
// 113.5 (squarings at 0.75; tools/gpu notes in DESIGN.md section 9), and k_ml_combine_d
// multiplies the 4 values.  Event values are read as repacked limbs (an Fp* scalar each; the
// final exponentiation removes them); every part is conj'd (conj is a field automorphism).
struct HornerParts {
  int n;
  int b[8];  // part p covers events [b[p], b[p + 1])
};
constexpr HornerParts kHornerParts4 = {4, {0, 7, 18, 36, 68, 68, 68, 68}};
constexpr HornerParts kHornerParts1 = {1, {0, 68, 68, 68, 68, 68, 68, 68}};

__global__ void __launch_bounds__(w12d::THREADS) k_ml_horner_d(const fp12 *V, uint32_t nseg,
                                                               fp12 *out, const uint32_t *lim,
                                                               uint32_t base, HornerParts hp) {
  __shared__ __attribute__((aligned(16))) uint32_t ev[ML_EVENTS * w12d::IMG], acc[w12d::IMG],
      ws[w12d::WS];
  const uint32_t s = blockIdx.x, part = blockIdx.y;
  if (lim && base + s >= *lim) return;  // block-uniform
  const int e0 = hp.b[part], e1 = hp.b[part + 1];
  w12d::Eng e;
  w12d::begin(e, ws);
  for (uint32_t q = e.row; q < (uint32_t)(e1 - e0) * 12; q += w12d::ROWS) {
    const uint32_t ev_i = q / 12, c = q % 12;
    const uint32_t *w = reinterpret_cast<const uint32_t *>(V + (size_t)(e0 + ev_i) * nseg + s) + 12 * c;
    ev[ev_i * w12d::IMG + 16 * c + e.j] = dfp::from_words_scaled(w);
  }
  __syncthreads();
  w12d::copy(e, acc, ev);
  for (int k = e0 + 1; k < e1; k++) {
    if (ev_is_dbl(k)) w12d::sqr(e, acc, acc);
    w12d::mul(e, acc, acc, ev + (k - e0) * w12d::IMG);
  }
  for (int k = e1; k < ML_EVENTS; k++)
    if (ev_is_dbl(k)) w12d::sqr(e, acc, acc);
  w12d::conj(e, acc, acc);
  w12d::store_words(e, reinterpret_cast<uint32_t *>(out + (size_t)part * nseg + s), acc);
}
// partial[s] = prod_p parts[p][s] (row engine; canonical words out)
__global__ void __launch_bounds__(w12d::THREADS) k_ml_combine_d(const fp12 *parts, uint32_t nparts,
                                                                uint32_t nseg, fp12 *partial,
                                                                const uint32_t *lim, uint32_t base) {
  __shared__ __attribute__((aligned(16))) uint32_t acc[w12d::IMG], tmp[w12d::IMG], ws[w12d::WS];
  const uint32_t s = blockIdx.x;
  if (lim && base + s >= *lim) return;  // block-uniform
  w12d::Eng e;
  w12d::begin(e, ws);
  w12d::load_scaled(e, acc, reinterpret_cast<const uint32_t *>(parts + s));
  for (uint32_t p = 1; p < nparts; p++) {
    w12d::load_scaled(e, tmp, reinterpret_cast<const uint32_t *>(parts + (size_t)p * nseg + s));
    w12d::mul(e, acc, acc, tmp);
  }
  w12d::store_words(e, reinterpret_cast<uint32_t *>(partial + s), acc);
}

// segments up to this many take the row-distributed (latency) form
constexpr uint32_t kHornerRowsMaxSegs = 64;

void launch_ml_horner(hipStream_t st, const fp12 *V, uint32_t nseg, fp12 *partial,
                      const uint32_t *lim, uint32_t base, fp12 *tmp) {
  if (!nseg) return;
  if (nseg <= kHornerRowsMaxSegs && tmp) {
    k_ml_horner_d<<<dim3(nseg, kHornerParts4.n), w12d::THREADS, 0, st>>>(V, nseg, tmp, lim, base, kHornerParts4);
    k_ml_combine_d<<<nseg, w12d::THREADS, 0, st>>>(tmp, kHornerParts4.n, nseg, partial, lim, base);
  } else if (nseg <= kHornerRowsMaxSegs) {
    k_ml_horner_d<<<dim3(nseg, 1), w12d::THREADS, 0, st>>>(V, nseg, partial, lim, base, kHornerParts1);
  } else {
    k_ml_horner<<<nseg, 64, 0, st>>>(V, nseg, partial, lim, base);
  }
}

}  // namespace gbls
