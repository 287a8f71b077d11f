// Microbenchmark: latency of one wave-cooperative Fp12 product (bls_wave12.h) and of
// each of its rounds, versus a plain single-lane Fp-mul chain.  One 64-thread block;
// timestamps from s_memtime (clock64), reported in shader cycles per operation.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I grandine_amd/csrc \
//         tools/ubench/w12_bench.hip -o tools/ubench/w12_bench
#include <hip/hip_runtime.h>
#include <stdio.h>

#include "bls_wave12.h"

using namespace gbls;

constexpr int ITERS = 256;

__global__ void __launch_bounds__(64) k_bench(const uint32_t *in, uint64_t *out, uint32_t *sink) {
  W12_SHARED uint32_t a[W12_WORDS], b[W12_WORDS], ws[W12_WS_WORDS];
  int lane = threadIdx.x;
  w12_plan pl;
  w12_begin(pl, ws);
  for (int i = lane; i < W12_WORDS; i += 64) {
    a[i] = in[i];
    b[i] = in[W12_WORDS + i];
  }
  __syncthreads();
  uint64_t t_mul = 0, t_p1 = 0, t_p2 = 0, t_p3 = 0;
  uint64_t r0 = __builtin_amdgcn_s_memrealtime();
  uint64_t t0 = clock64();
  for (int it = 0; it < ITERS; it++) w12_mul(pl, a, a, b, ws);
  uint64_t t1 = clock64();
  uint64_t r1 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < ITERS; it++) {
    uint64_t s0 = clock64();
    w12_r_mul(lane, pl, a, b, ws);
    __syncthreads();
    uint64_t s1 = clock64();
    w12_r_post1(lane, pl, ws);
    __syncthreads();
    uint64_t s2 = clock64();
    w12_r_post2(lane, pl, ws);
    __syncthreads();
    uint64_t s3 = clock64();
    w12_r_post3(lane, pl, ws, a);
    __syncthreads();
    uint64_t s4 = clock64();
    t_mul += s1 - s0;
    t_p1 += s2 - s1;
    t_p2 += s3 - s2;
    t_p3 += s4 - s3;
  }
  // single-lane Fp chain
  fp x, y;
  ld_fp(x, a + 12 * (lane % 12));
  ld_fp(y, b + 12 * (lane % 12));
  uint64_t u0 = clock64();
  for (int it = 0; it < ITERS; it++) fp_mul(x, x, y);
  uint64_t u1 = clock64();
  st_fp(sink + 12 * lane, x);
  if (lane == 0) {
    out[0] = (t1 - t0) / ITERS;
    out[1] = t_mul / ITERS;
    out[2] = t_p1 / ITERS;
    out[3] = t_p2 / ITERS;
    out[4] = t_p3 / ITERS;
    out[5] = (u1 - u0) / ITERS;
    out[6] = t1 - t0;
    out[7] = r1 - r0;  // 100 MHz ticks
  }
  for (int i = lane; i < W12_WORDS; i += 64) sink[64 * 12 + i] = a[i];
}

int main() {
  uint32_t h[2 * W12_WORDS];
  for (int i = 0; i < 2 * W12_WORDS; i++) h[i] = (i % 12 == 11) ? 0x01234567u : 0x9e3779b9u * (i + 1);
  uint32_t *din, *sink;
  uint64_t *dout;
  hipMalloc(&din, sizeof h);
  hipMalloc(&dout, 8 * 8);
  hipMalloc(&sink, 4 * (64 * 12 + W12_WORDS));
  hipMemcpy(din, h, sizeof h, hipMemcpyHostToDevice);
  uint64_t o[8] = {0};
  for (int rep = 0; rep < 3; rep++) {
    k_bench<<<1, 64>>>(din, dout, sink);
    if (hipDeviceSynchronize() != hipSuccess) {
      printf("kernel failed\n");
      return 1;
    }
  }
  hipMemcpy(o, dout, 8 * 8, hipMemcpyDeviceToHost);
  double ghz = (double)o[6] / ((double)o[7] * 10.0);  // cycles per ns
  printf("shader clock %.2f GHz\n", ghz);
  printf("cycles per op: w12_mul %llu (%.2f us) | mul-round %llu post1 %llu post2 %llu post3 %llu | "
         "fp_mul chain %llu (%.2f us)\n",
         (unsigned long long)o[0], o[0] / ghz / 1e3, (unsigned long long)o[1], (unsigned long long)o[2],
         (unsigned long long)o[3], (unsigned long long)o[4], (unsigned long long)o[5], o[5] / ghz / 1e3);
  return 0;
}
