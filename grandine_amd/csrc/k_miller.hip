// gfx950 kernels: the batch Miller product as a tree (bls_pairing.h header comment).
//   k_ml_leaf   lane per (event e, couple of pairs): line_e(P_a) * line_e(P_b)
//               (two sparse evaluations, 6 Fp2 products) -> dense Fp12
//   k_ml_reduce wave per (event, group of <= 4 values of one segment): wave-cooperative
//               Fp12 products (bls_wave12.h)
//   k_ml_horner wave per segment: Horner over the 68 events, then conj (x < 0)
#include "bls_wave12.h"
#include "gbls_common.h"

namespace gbls {

// grid (ceil(ncouple / 64), 68)
__global__ void __launch_bounds__(WG) k_ml_leaf(const uint32_t *L, uint32_t np, const g1s *P,
                                                const uint32_t *couples, uint32_t ncouple,
                                                fp12 *V0) {
  uint32_t c = blockIdx.x * WG + threadIdx.x;
  int e = blockIdx.y;
  if (c >= ncouple) return;
  uint32_t pa = couples[2 * c], pb = couples[2 * c + 1];
  fp2 L0, L2, L3;
  sp034 sa, sb;
  line_get(L, np, pa, e, L0, L2, L3);
  g1s Pa = P[pa];
  line_eval_s(sa, L0, L2, L3, Pa);
  fp12 r;
  if (pb != NONE) {
    line_get(L, np, pb, e, L0, L2, L3);
    g1s Pb = P[pb];
    line_eval_s(sb, L0, L2, L3, Pb);
    sp_mul_sp(r, sa, sb);
  } else {
    sp_to_fp12(r, sa);
  }
  V0[(size_t)e * ncouple + c] = r;
}

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
__global__ void __launch_bounds__(64) k_ml_horner(const fp12 *V, uint32_t nseg, fp12 *partial) {
  W12_SHARED uint32_t acc[W12_WORDS], tmp[W12_WORDS], ws[W12_WS_WORDS];
  w12_plan pl;
  w12_begin(pl, ws);
  uint32_t s = blockIdx.x;
  w12_load(acc, V + s);
  for (int e = 1; e < ML_EVENTS; e++) {
    if (ev_is_dbl(e)) w12_mul(pl, acc, acc, acc, ws);
    w12_load(tmp, V + (size_t)e * nseg + s);
    w12_mul(pl, acc, acc, tmp, ws);
  }
  w12_conj(acc, acc);
  w12_store(partial + s, acc);
}

void launch_ml_leaf(hipStream_t st, const uint32_t *lines, uint32_t np, const g1s *P,
                    const uint32_t *couples, uint32_t ncouple, fp12 *V0) {
  dim3 grid(nblk(ncouple), ML_EVENTS);
  if (ncouple) k_ml_leaf<<<grid, WG, 0, st>>>(lines, np, P, couples, ncouple, V0);
}
void launch_ml_reduce(hipStream_t st, const fp12 *Vin, uint32_t nin, const uint32_t *red,
                      uint32_t nout, fp12 *Vout) {
  dim3 grid(nout, ML_EVENTS);
  if (nout) k_ml_reduce<<<grid, 64, 0, st>>>(Vin, nin, red, nout, Vout);
}
void launch_ml_horner(hipStream_t st, const fp12 *V, uint32_t nseg, fp12 *partial) {
  if (nseg) k_ml_horner<<<nseg, 64, 0, st>>>(V, nseg, partial);
}

}  // namespace gbls
