// Microbenchmarks for the field-arithmetic design decision (gfx950):
//   mad64 peak, fp64 FMA peak, and Fp (381-bit Montgomery) multiply throughput of
//   several formulations / occupancies.  Standalone: hipcc -O3 --offload-arch=gfx950.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include "../../grandine_amd/csrc/bls_constants.h"

using namespace gbls;
#define DI __device__ __forceinline__

struct fpv { uint32_t l[12]; };

// ---- variant R: current engine (outer loop rolled, b rotated)
DI void mul_rolled(fpv &r, const fpv &a, const fpv &b) {
  uint32_t t[12], bb[12];
#pragma unroll
  for (int j = 0; j < 12; j++) { t[j] = 0; bb[j] = b.l[j]; }
#pragma unroll 1
  for (int i = 0; i < 12; i++) {
    const uint32_t bi = bb[0];
#pragma unroll
    for (int j = 0; j < 11; j++) bb[j] = bb[j + 1];
    uint64_t s = (uint64_t)a.l[0] * bi + t[0];
    uint32_t A = (uint32_t)(s >> 32), t0 = (uint32_t)s, m = t0 * k::PINV;
    uint64_t s2 = (uint64_t)m * k::P[0] + t0;
    uint32_t C = (uint32_t)(s2 >> 32);
#pragma unroll
    for (int j = 1; j < 12; j++) {
      s = (uint64_t)a.l[j] * bi + t[j] + A; A = (uint32_t)(s >> 32);
      s2 = (uint64_t)m * k::P[j] + (uint32_t)s + C; C = (uint32_t)(s2 >> 32);
      t[j - 1] = (uint32_t)s2;
    }
    t[11] = A + C;
  }
  uint32_t u[12], br = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) { uint64_t d = (uint64_t)t[i] - k::P[i] - br; u[i] = (uint32_t)d; br = (uint32_t)(d >> 63); }
  uint32_t msk = 0u - br;
#pragma unroll
  for (int i = 0; i < 12; i++) r.l[i] = (u[i] & ~msk) | (t[i] & msk);
}

// ---- variant U: fully unrolled CIOS
DI void mul_unrolled(fpv &r, const fpv &a, const fpv &b) {
  uint32_t t[12];
#pragma unroll
  for (int j = 0; j < 12; j++) t[j] = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    const uint32_t bi = b.l[i];
    uint64_t s = (uint64_t)a.l[0] * bi + t[0];
    uint32_t A = (uint32_t)(s >> 32), t0 = (uint32_t)s, m = t0 * k::PINV;
    uint64_t s2 = (uint64_t)m * k::P[0] + t0;
    uint32_t C = (uint32_t)(s2 >> 32);
#pragma unroll
    for (int j = 1; j < 12; j++) {
      s = (uint64_t)a.l[j] * bi + t[j] + A; A = (uint32_t)(s >> 32);
      s2 = (uint64_t)m * k::P[j] + (uint32_t)s + C; C = (uint32_t)(s2 >> 32);
      t[j - 1] = (uint32_t)s2;
    }
    t[11] = A + C;
  }
  uint32_t u[12], br = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) { uint64_t d = (uint64_t)t[i] - k::P[i] - br; u[i] = (uint32_t)d; br = (uint32_t)(d >> 63); }
  uint32_t msk = 0u - br;
#pragma unroll
  for (int i = 0; i < 12; i++) r.l[i] = (u[i] & ~msk) | (t[i] & msk);
}

// ---- variant M: mad64 with 64-bit addend carrying (t_j + carry) via the mad's own addend
// s = a_j*b_i + (t_j | A<<32)?  no: use two chains with explicit 64-bit accumulate
DI uint64_t mad64(uint32_t a, uint32_t b, uint64_t c) { return (uint64_t)a * b + c; }
DI void mul_mad(fpv &r, const fpv &a, const fpv &b) {
  uint32_t t[13];
#pragma unroll
  for (int j = 0; j < 13; j++) t[j] = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    const uint32_t bi = b.l[i];
    // t += a * bi   (carry chain through the mad's 64-bit addend)
    uint64_t acc = 0;
#pragma unroll
    for (int j = 0; j < 12; j++) {
      acc = mad64(a.l[j], bi, (acc >> 32) + t[j]);
      t[j] = (uint32_t)acc;
    }
    uint64_t top = (uint64_t)t[12] + (acc >> 32);
    // reduce: t = (t + m p) / 2^32
    uint32_t m = t[0] * k::PINV;
    acc = mad64(m, k::P[0], t[0]);
#pragma unroll
    for (int j = 1; j < 12; j++) {
      acc = mad64(m, k::P[j], (acc >> 32) + t[j]);
      t[j - 1] = (uint32_t)acc;
    }
    top += acc >> 32;
    t[11] = (uint32_t)top;
    t[12] = (uint32_t)(top >> 32);
  }
  uint32_t u[12], br = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) { uint64_t d = (uint64_t)t[i] - k::P[i] - br; u[i] = (uint32_t)d; br = (uint32_t)(d >> 63); }
  uint32_t msk = 0u - br;
#pragma unroll
  for (int i = 0; i < 12; i++) r.l[i] = (u[i] & ~msk) | (t[i] & msk);
}


// ---- variant F: product-scanning Montgomery (FIPS), 96-bit column accumulator,
// carry-out of v_mad_u64_u32 folded into the third word (inline asm)
DI void mac_asm(uint64_t &acc, uint32_t &c2, uint32_t a, uint32_t b) {
  asm("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
      : "+v"(acc), "+v"(c2) : "v"(a), "v"(b) : "vcc");
}
DI void mac_c(uint64_t &acc, uint32_t &c2, uint32_t a, uint32_t b) {
  uint64_t p = (uint64_t)a * b;
  acc += p;
  c2 += (acc < p);
}
template <bool ASM>
DI void mul_fips(fpv &r, const fpv &a, const fpv &b) {
  uint32_t m[12], t[12];
  uint64_t acc = 0;
  uint32_t c2 = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) {
#pragma unroll
    for (int j = 0; j < i; j++) {
      if (ASM) { mac_asm(acc, c2, a.l[j], b.l[i - j]); mac_asm(acc, c2, m[j], k::P[i - j]); }
      else { mac_c(acc, c2, a.l[j], b.l[i - j]); mac_c(acc, c2, m[j], k::P[i - j]); }
    }
    if (ASM) mac_asm(acc, c2, a.l[i], b.l[0]); else mac_c(acc, c2, a.l[i], b.l[0]);
    m[i] = (uint32_t)acc * k::PINV;
    if (ASM) mac_asm(acc, c2, m[i], k::P[0]); else mac_c(acc, c2, m[i], k::P[0]);
    acc = (acc >> 32) | ((uint64_t)c2 << 32);
    c2 = 0;
  }
#pragma unroll
  for (int i = 12; i < 24; i++) {
#pragma unroll
    for (int j = i - 11; j < 12; j++) {
      if (ASM) { mac_asm(acc, c2, a.l[j], b.l[i - j]); mac_asm(acc, c2, m[j], k::P[i - j]); }
      else { mac_c(acc, c2, a.l[j], b.l[i - j]); mac_c(acc, c2, m[j], k::P[i - j]); }
    }
    t[i - 12] = (uint32_t)acc;
    acc = (acc >> 32) | ((uint64_t)c2 << 32);
    c2 = 0;
  }
  uint32_t u[12], br = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) { uint64_t d = (uint64_t)t[i] - k::P[i] - br; u[i] = (uint32_t)d; br = (uint32_t)(d >> 63); }
  uint32_t msk = 0u - br;
#pragma unroll
  for (int i = 0; i < 12; i++) r.l[i] = (u[i] & ~msk) | (t[i] & msk);
}

template <int V> DI void fmul(fpv &r, const fpv &a, const fpv &b) {
  if (V == 0) mul_rolled(r, a, b);
  else if (V == 1) mul_unrolled(r, a, b);
  else if (V == 2) mul_mad(r, a, b);
  else if (V == 3) mul_fips<true>(r, a, b);
  else mul_fips<false>(r, a, b);
}

// CH independent chains per lane, iters squarings+mults each
template <int V, int CH, int WPS>
__global__ void __launch_bounds__(256, WPS) k_fpmul(uint32_t *out, uint32_t iters, uint32_t seed) {
  fpv x[CH], y;
#pragma unroll
  for (int i = 0; i < 12; i++) y.l[i] = (seed * 2654435761u + i * 97 + threadIdx.x) & 0x0fffffff;
#pragma unroll
  for (int c = 0; c < CH; c++)
#pragma unroll
    for (int i = 0; i < 12; i++) x[c].l[i] = (seed + c * 7919u + i * 31 + blockIdx.x) & 0x0fffffff;
  for (uint32_t it = 0; it < iters; it++) {
#pragma unroll
    for (int c = 0; c < CH; c++) fmul<V>(x[c], x[c], y);
  }
  uint32_t acc = 0;
#pragma unroll
  for (int c = 0; c < CH; c++)
#pragma unroll
    for (int i = 0; i < 12; i++) acc ^= x[c].l[i];
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

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

__global__ void __launch_bounds__(256) k_fma64_peak(double *sink, uint32_t iters, double seed) {
  double acc[8];
  double a = seed + threadIdx.x * 1e-9, b = 0.999999;
#pragma unroll
  for (int j = 0; j < 8; j++) acc[j] = a + j;
  for (uint32_t it = 0; it < iters; it++) {
#pragma unroll
    for (int j = 0; j < 8; j++) acc[j] = fma(acc[j], b, a);
  }
  double x = 0;
#pragma unroll
  for (int j = 0; j < 8; j++) x += acc[j];
  if (x == 0.123456) sink[0] = x;
}

__global__ void __launch_bounds__(256) k_mullo_peak(uint32_t *sink, uint32_t iters, uint32_t seed) {
  uint32_t acc[8];
  uint32_t a = seed ^ threadIdx.x;
#pragma unroll
  for (int j = 0; j < 8; j++) acc[j] = a + j;
  for (uint32_t it = 0; it < iters; it++) {
#pragma unroll
    for (int j = 0; j < 8; j++) acc[j] = acc[j] * acc[j] + a;
  }
  uint32_t x = 0;
#pragma unroll
  for (int j = 0; j < 8; j++) x ^= acc[j];
  if (x == 0x12345) sink[0] = x;
}

static float timeit(void (*launch)(hipStream_t), hipStream_t s) {
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  launch(s);
  hipEventRecord(a, s);
  launch(s);
  hipEventRecord(b, s);
  hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  hipEventDestroy(a); hipEventDestroy(b);
  return ms;
}

static void *g_sink;
static const unsigned BLOCKS = 256 * 16;
template <int V, int CH, int WPS>
static void run_fpmul(const char *name) {
  const uint32_t iters = 256;
  auto L = [](hipStream_t s) { k_fpmul<V, CH, WPS><<<BLOCKS, 256, 0, s>>>((uint32_t *)g_sink, 256, 3); };
  float ms = timeit(L, 0);
  double muls = (double)BLOCKS * 256 * iters * CH;
  printf("fpmul %-10s CH=%d WPS=%d: %.3f ms  %.3e Fp-mul/s  (= %.3e mad64-equiv/s at 288/mul)\n", name, CH, WPS, ms,
         muls / (ms * 1e-3), muls * 288 / (ms * 1e-3));
}

int main() {
  hipMalloc(&g_sink, (size_t)BLOCKS * 256 * 8);
  {
    auto L = [](hipStream_t s) { k_mad_peak<<<2048, 256, 0, s>>>((uint64_t *)g_sink, 4096, 7); };
    float ms = timeit(L, 0);
    printf("mad64 peak: %.3e mad/s (%.3f ms)\n", 2048.0 * 256 * 4096 * 16 / (ms * 1e-3), ms);
  }
  {
    auto L = [](hipStream_t s) { k_fma64_peak<<<2048, 256, 0, s>>>((double *)g_sink, 4096, 1.5); };
    float ms = timeit(L, 0);
    printf("fma64 peak: %.3e fma/s (%.3f ms)\n", 2048.0 * 256 * 4096 * 8 / (ms * 1e-3), ms);
  }
  {
    auto L = [](hipStream_t s) { k_mullo_peak<<<2048, 256, 0, s>>>((uint32_t *)g_sink, 4096, 1); };
    float ms = timeit(L, 0);
    printf("mul_lo_u32+add peak: %.3e /s (%.3f ms)\n", 2048.0 * 256 * 4096 * 8 / (ms * 1e-3), ms);
  }
  run_fpmul<0, 1, 1>("rolled");
  run_fpmul<0, 2, 1>("rolled");
  run_fpmul<0, 1, 2>("rolled");
  run_fpmul<0, 2, 2>("rolled");
  run_fpmul<0, 1, 4>("rolled");
  run_fpmul<1, 1, 1>("unrolled");
  run_fpmul<1, 2, 1>("unrolled");
  run_fpmul<1, 1, 2>("unrolled");
  run_fpmul<1, 2, 2>("unrolled");
  run_fpmul<1, 1, 4>("unrolled");
  run_fpmul<2, 1, 1>("mad");
  run_fpmul<2, 2, 1>("mad");
  run_fpmul<2, 1, 2>("mad");
  run_fpmul<2, 2, 2>("mad");
  run_fpmul<2, 1, 4>("mad");
  run_fpmul<3, 1, 1>("fips-asm");
  run_fpmul<3, 2, 1>("fips-asm");
  run_fpmul<3, 1, 2>("fips-asm");
  run_fpmul<3, 2, 2>("fips-asm");
  run_fpmul<3, 1, 4>("fips-asm");
  run_fpmul<3, 1, 8>("fips-asm");
  run_fpmul<4, 1, 1>("fips-c");
  run_fpmul<4, 1, 2>("fips-c");
  run_fpmul<4, 1, 4>("fips-c");
  run_fpmul<1, 1, 8>("unrolled");
  hipError_t e = hipDeviceSynchronize();
  printf("status %s\n", hipGetErrorString(e));
  return 0;
}
