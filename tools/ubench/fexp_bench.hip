// Microbenchmark: where the final exponentiation's time goes (k_fexp.hip): cycles of
// one w12_mul, one cyclotomic squaring, the single-lane Fp12 inversion, one exponentiation
// by x and the whole chain, on one 64-lane workgroup (s_memtime / clock64).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I grandine_amd/csrc \
//         tools/ubench/fexp_bench.hip -o tools/ubench/fexp_bench
#include <hip/hip_runtime.h>
#include <stdio.h>

#include "bls_wave12.h"

using namespace gbls;

constexpr int ITERS = 64;

__global__ void __launch_bounds__(64) k_bench(const uint32_t *in, uint64_t *out, uint32_t *sink) {
  W12_SHARED uint32_t a[W12_WORDS], b[W12_WORDS], c[W12_WORDS], ws[W12_WS_WORDS];
  int lane = threadIdx.x;
  w12_plan pl;
  w12_begin(pl, ws);
  w12_cplan cp;
  w12_cplan_load(cp, lane);
  for (int i = lane; i < W12_WORDS; i += 64) {
    a[i] = in[i];
    b[i] = in[W12_WORDS + i];
  }
  __syncthreads();
  uint64_t t0 = clock64();
  for (int it = 0; it < ITERS; it++) w12_mul(pl, a, a, b, ws);
  uint64_t t1 = clock64();
  for (int it = 0; it < ITERS; it++) w12_cyc_sqr(cp, a, a, ws);
  uint64_t t2 = clock64();
  for (int it = 0; it < 4; it++) w12_inv(c, a);
  uint64_t t3 = clock64();
  w12_cyc_exp_x(pl, cp, c, a, ws);
  uint64_t t4 = clock64();
  uint64_t r0 = __builtin_amdgcn_s_memrealtime();
  uint64_t t5 = clock64();
  // the k_final_verdict chain
  w12_inv(c, a);
  w12_conj(b, a);
  w12_mul(pl, b, b, c, ws);
  w12_frob2(a, b);
  w12_mul(pl, a, a, b, ws);
  for (int k = 0; k < 5; k++) {
    w12_cyc_exp_x(pl, cp, c, a, ws);
    w12_mul(pl, a, c, b, ws);
  }
  uint64_t t6 = clock64();
  uint64_t r1 = __builtin_amdgcn_s_memrealtime();
  if (lane == 0) {
    out[0] = (t1 - t0) / ITERS;
    out[1] = (t2 - t1) / ITERS;
    out[2] = (t3 - t2) / 4;
    out[3] = t4 - t3;
    out[4] = t6 - t5;
    out[5] = r1 - r0;
  }
  for (int i = lane; i < W12_WORDS; i += 64) sink[i] = a[i] ^ c[i];
}

int main() {
  uint32_t h[2 * W12_WORDS];
  for (int i = 0; i < 2 * W12_WORDS; i++) h[i] = (i % 12 == 11) ? 0x01234567u : 0x9e3779b9u * (i + 1);
  uint32_t *din, *sink;
  uint64_t *dout;
  (void)hipMalloc(&din, sizeof h);
  (void)hipMalloc(&dout, 8 * 8);
  (void)hipMalloc(&sink, 4 * W12_WORDS);
  (void)hipMemcpy(din, h, sizeof h, hipMemcpyHostToDevice);
  uint64_t o[8] = {0};
  for (int rep = 0; rep < 3; rep++) {
    k_bench<<<1, 64>>>(din, dout, sink);
    if (hipDeviceSynchronize() != hipSuccess) {
      printf("kernel failed\n");
      return 1;
    }
  }
  (void)hipMemcpy(o, dout, 8 * 8, hipMemcpyDeviceToHost);
  double ghz = (double)o[4] / ((double)o[5] * 10.0);
  printf("shader clock %.2f GHz\n", ghz);
  printf("cycles: w12_mul %llu | cyc_sqr %llu | fp12 inv (lane 0) %llu | exp_by_x %llu | chain %llu (%.3f ms)\n",
         (unsigned long long)o[0], (unsigned long long)o[1], (unsigned long long)o[2],
         (unsigned long long)o[3], (unsigned long long)o[4], o[4] / ghz / 1e6);
  return 0;
}
