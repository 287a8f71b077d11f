// Occupancy microbenchmark: the engine's own device Montgomery product (bls_field.h,
// fp_mul_dev from tools/gen_fpmul.py) in dependent chains, launched as exactly W waves of
// 64 lanes on the 1024 SIMDs of an MI355X, so that 1, 2 or 4 waves share a SIMD (the
// kernels of the engine run at one wave per SIMD: 256 VGPRs + AGPRs).  Also one wave per
// SIMD with 2 independent chains per lane (instruction-level parallelism).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o occ_bench occ_bench.hip
#include <cstdio>

#include "../../grandine_amd/csrc/bls_field.h"

using namespace gbls;

template <int CH>
__global__ void __launch_bounds__(64) k_chain(uint32_t *out, uint32_t iters, uint32_t seed) {
  fp x[CH], y;
#pragma unroll
  for (int i = 0; i < 12; i++) y.l[i] = (seed * 2654435761u + i * 97 + threadIdx.x) & 0x0fffffff;
#pragma unroll
  for (int c = 0; c < CH; c++)
#pragma unroll
    for (int i = 0; i < 12; i++) x[c].l[i] = (seed + c * 7919u + i * 31 + blockIdx.x) & 0x0fffffff;
  for (uint32_t it = 0; it < iters; it++) {
#pragma unroll
    for (int c = 0; c < CH; c++) fp_mul(x[c], x[c], y);
  }
  uint32_t acc = 0;
#pragma unroll
  for (int c = 0; c < CH; c++)
#pragma unroll
    for (int i = 0; i < 12; i++) acc ^= x[c].l[i];
  out[blockIdx.x * 64 + threadIdx.x] = acc;
}

template <int CH>
static void run(uint32_t *sink, int waves, uint32_t iters) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  k_chain<CH><<<waves, 64>>>(sink, iters, 1);
  hipEventRecord(a);
  k_chain<CH><<<waves, 64>>>(sink, iters, 3);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  double muls = (double)waves * 64 * iters * CH;
  printf("waves=%5d (%.0f per SIMD) chains/lane=%d: %8.3f ms  %.3e Fp-mul/s  per-lane latency %.3f us/mul\n",
         waves, waves / 1024.0, CH, ms, muls / (ms * 1e-3), ms * 1e3 / (iters * CH));
}

int main() {
  uint32_t *sink;
  hipMalloc(&sink, 8192 * 64 * 4);
  const uint32_t it = 2000;
  run<1>(sink, 1024, it);
  run<1>(sink, 2048, it);
  run<1>(sink, 4096, it);
  run<2>(sink, 1024, it / 2);
  run<2>(sink, 2048, it / 2);
  run<1>(sink, 1024, it);
  printf("status %s\n", hipGetErrorString(hipDeviceSynchronize()));
  return 0;
}
