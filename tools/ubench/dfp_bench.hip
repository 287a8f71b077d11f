// Row-distributed Fp product (bls_dfp.h) on MI355X: bit-exactness against the engine's
// one-lane product (bls_field.h fp_mul) on random operands and long dependent chains, and
// the latency of a dependent chain of products per row vs per lane.
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -o tools/ubench/_bin/dfp_bench tools/ubench/dfp_bench.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "../../grandine_amd/csrc/gbls_common.h"
#include "../../grandine_amd/csrc/bls_dfp.h"

using namespace gbls;

// one row per (a, b) pair: c = a b (engine and row forms) and a chain x <- x^2 b, K steps
__global__ void __launch_bounds__(256) k_check(const fp *A, const fp *B, uint32_t n, uint32_t K,
                                               fp *out_eng, fp *out_row) {
  dfp::Tabs t;
  dfp::load_tabs(t);
  const uint32_t row = (blockIdx.x * blockDim.x + threadIdx.x) >> 4;
  if (row >= n) return;
  const fp a = A[row], b = B[row];
  // row form
  uint32_t xa = dfp::from_words(a.l, t), xb = dfp::from_words(b.l, t);
  uint32_t x = dfp::mul(xa, xb, t);
  for (uint32_t k = 0; k < K; k++) x = dfp::mul(dfp::mul(x, x, t), xb, t);
  __shared__ uint32_t w[16][12];
  dfp::to_words(w[(threadIdx.x >> 4) & 15], x, t);
  __syncthreads();
  if ((threadIdx.x & 15) == 0) {
    fp e;
    fp_mul(e, a, b);
    for (uint32_t k = 0; k < K; k++) {
      fp_mul(e, e, e);
      fp_mul(e, e, b);
    }
    out_eng[row] = e;
    fp r;
    for (int i = 0; i < 12; i++) r.l[i] = w[(threadIdx.x >> 4) & 15][i];
    out_row[row] = r;
  }
}

// latency: one row (16 lanes) or one lane runs K dependent products
__global__ void __launch_bounds__(64) k_lat_row(const fp *A, uint32_t K, fp *out, uint64_t *cyc) {
  dfp::Tabs t;
  dfp::load_tabs(t);
  uint32_t x = dfp::from_words(A[blockIdx.x].l, t), y = x;
  uint64_t c0 = wall_clock64();
  for (uint32_t k = 0; k < K; k++) x = dfp::mul(x, y, t);
  uint64_t c1 = wall_clock64();
  __shared__ uint32_t w[4][12];
  dfp::to_words(w[threadIdx.x >> 4], x, t);
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 0; i < 12; i++) out[blockIdx.x].l[i] = w[0][i];
    cyc[blockIdx.x] = c1 - c0;
  }
}
__global__ void __launch_bounds__(64) k_lat_lane(const fp *A, uint32_t K, fp *out, uint64_t *cyc) {
  fp x = A[blockIdx.x], y = x;
  uint64_t c0 = wall_clock64();
  for (uint32_t k = 0; k < K; k++) fp_mul(x, x, y);
  uint64_t c1 = wall_clock64();
  if (threadIdx.x == 0) {
    out[blockIdx.x] = x;
    cyc[blockIdx.x] = c1 - c0;
  }
}

static const uint32_t P32[12] = {0xffffaaab, 0xb9feffff, 0xb153ffff, 0x1eabfffe, 0xf6b0f624, 0x6730d2a0,
                                 0xf38512bf, 0x64774b84, 0x434bacd7, 0x4b1ba7b6, 0x397fe69a, 0x1a0111ea};
static uint64_t rs = 88172645463325252ull;
static uint32_t rnd() {
  rs ^= rs << 13;
  rs ^= rs >> 7;
  rs ^= rs << 17;
  return (uint32_t)rs;
}
static void rand_fp(fp &x) {  // uniform-ish below p: top word reduced
  for (int i = 0; i < 12; i++) x.l[i] = rnd();
  x.l[11] %= 0x1a0111ea;
}

#define CK(x)                                                    \
  do {                                                           \
    hipError_t e_ = (x);                                         \
    if (e_ != hipSuccess) {                                      \
      printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); \
      return 1;                                                  \
    }                                                            \
  } while (0)

int main() {
  const uint32_t n = 4096;
  fp *hA = (fp *)malloc(n * sizeof(fp)), *hB = (fp *)malloc(n * sizeof(fp));
  for (uint32_t i = 0; i < n; i++) {
    rand_fp(hA[i]);
    rand_fp(hB[i]);
  }
  // edge operands: 0, 1 (raw), p - 1, max
  for (int i = 0; i < 12; i++) {
    hA[0].l[i] = 0;
    hA[1].l[i] = i == 0;
    hA[2].l[i] = P32[i] - (i == 0);
    hB[2].l[i] = P32[i] - (i == 0);
  }
  fp *dA, *dB, *dE, *dR;
  uint64_t *dc;
  CK(hipMalloc(&dA, n * sizeof(fp)));
  CK(hipMalloc(&dB, n * sizeof(fp)));
  CK(hipMalloc(&dE, n * sizeof(fp)));
  CK(hipMalloc(&dR, n * sizeof(fp)));
  CK(hipMalloc(&dc, 1024 * 8));
  CK(hipMemcpy(dA, hA, n * sizeof(fp), hipMemcpyHostToDevice));
  CK(hipMemcpy(dB, hB, n * sizeof(fp), hipMemcpyHostToDevice));
  fp *hE = (fp *)malloc(n * sizeof(fp)), *hR = (fp *)malloc(n * sizeof(fp));
  for (uint32_t K : {0u, 1u, 64u}) {
    k_check<<<n * 16 / 256, 256>>>(dA, dB, n, K, dE, dR);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(hE, dE, n * sizeof(fp), hipMemcpyDeviceToHost));
    CK(hipMemcpy(hR, dR, n * sizeof(fp), hipMemcpyDeviceToHost));
    uint32_t bad = 0;
    for (uint32_t i = 0; i < n; i++)
      for (int l = 0; l < 12; l++)
        if (hE[i].l[l] != hR[i].l[l]) {
          if (bad < 3) printf("mismatch K=%u i=%u limb %d: %08x vs %08x\n", K, i, l, hE[i].l[l], hR[i].l[l]);
          bad++;
          break;
        }
    printf("check K=%u: %u / %u rows differ\n", K, bad, n);
    if (bad) return 2;
  }
  // latency, one block per CU-ish (256 blocks): each block = one wave = 4 rows
  const uint32_t K = 4096;
  uint64_t hc[256];
  for (int rep = 0; rep < 2; rep++) {
    k_lat_row<<<256, 64>>>(dA, K, dR, dc);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(hc, dc, 256 * 8, hipMemcpyDeviceToHost));
    double s = 0;
    for (int i = 0; i < 256; i++) s += hc[i];
    printf("row product: %.1f ns per dependent product (wall clock 100 MHz ticks)\n", s / 256 / K * 10.0);
    k_lat_lane<<<256, 64>>>(dA, K, dE, dc);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(hc, dc, 256 * 8, hipMemcpyDeviceToHost));
    s = 0;
    for (int i = 0; i < 256; i++) s += hc[i];
    printf("lane product: %.1f ns per dependent product\n", s / 256 / K * 10.0);
  }
  return 0;
}
