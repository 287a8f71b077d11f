// Radix-2^28 Montgomery product microbenchmark (next-round field-layer candidate).
// 381-bit p in 14 limbs of 28 bits, R = 2^392: a column of the product-scanning
// Montgomery product holds at most 28 (42 for a dual product) terms < 2^56, so a plain
// 64-bit accumulator needs no carry word: one v_mad_u64_u32 per term instead of the
// engine's mad + addc pair (bls_fpmul_gen.h), 392 terms against 288 pairs.  R/p ~ 2^11.3,
// so inputs < 2p give outputs < 1.002 p and no final subtraction is needed.
// Modes: rate (dependent chains, W waves, as occ_bench.hip) and check (prints a, b, a*b/R for
// tools/ubench/r28_check.py).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o r28_bench r28_bench.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstring>

#include "../../grandine_amd/csrc/bls_field.h"
#include "../../grandine_amd/csrc/bls_field28.h"

// the layer under test: grandine_amd/csrc/bls_field28.h (mul28<NACC> below is the
// accumulator-split experiment; the Fp2 chain runs the header's fe2_mul)
using f28 = gbls::r28::fe;
using f28x2 = gbls::r28::fe2;

#define P28_LIST                                                                               \
  0xfffaaab, 0xfefffff, 0x3ffffb9, 0xfffeb15, 0x6241eab, 0xa0f6b0f, 0xf6730d2, 0xf38512b,       \
      0x4774b84, 0x4bacd76, 0xba7b643, 0xe69a4b1, 0x1ea397f, 0x1a011
static constexpr uint32_t kPinv28 = 0xffcfffd;
static constexpr uint32_t kM28 = 0xfffffff;

// NACC independent accumulators per column (the terms alternate between them) to shorten
// the dependent mad chain; merged before the column's limb is taken.
template <int NACC>
__device__ __forceinline__ void mul28(f28 &r, const f28 &a, const f28 &b) {
  constexpr uint32_t P[14] = {P28_LIST};
  uint32_t m[14], t[14];
  uint64_t carry = 0;
#pragma unroll
  for (int k = 0; k < 27; k++) {
    uint64_t acc[NACC];
#pragma unroll
    for (int q = 0; q < NACC; q++) acc[q] = 0;
    acc[0] = carry;
    int n = 0;
#pragma unroll
    for (int i = 0; i < 14; i++) {
      const int j = k - i;
      if (j >= 0 && j < 14) acc[(n++) % NACC] += (uint64_t)a.l[i] * b.l[j];
    }
#pragma unroll
    for (int i = 0; i < 14; i++) {
      const int j = k - i;
      if (i < k && j >= 0 && j < 14) acc[(n++) % NACC] += (uint64_t)m[i] * P[j];
    }
#pragma unroll
    for (int q = 1; q < NACC; q++) acc[0] += acc[q];
    if (k < 14) {
      m[k] = ((uint32_t)acc[0] * kPinv28) & kM28;
      acc[0] += (uint64_t)m[k] * P[0];
      carry = acc[0] >> 28;
    } else {
      t[k - 14] = (uint32_t)acc[0] & kM28;
      carry = acc[0] >> 28;
    }
  }
  t[13] = (uint32_t)carry;
#pragma unroll
  for (int i = 0; i < 14; i++) r.l[i] = t[i];
}

__device__ __forceinline__ void fp2_mul28(f28x2 &r, const f28x2 &a, const f28x2 &b) {
  gbls::r28::fe2_mul(r, a, b);
}
__global__ void __launch_bounds__(64) k_chain2_28(uint32_t *out, uint32_t iters, uint32_t seed) {
  f28x2 x, y;
#pragma unroll
  for (int i = 0; i < 14; i++) {
    const uint32_t mk = i == 13 ? 0xffff : kM28;
    y.c0.l[i] = (seed * 2654435761u + i * 97 + threadIdx.x) & mk;
    y.c1.l[i] = (seed * 40503u + i * 13 + threadIdx.x) & mk;
    x.c0.l[i] = (seed + i * 31 + blockIdx.x) & mk;
    x.c1.l[i] = (seed + i * 57 + blockIdx.x) & mk;
  }
  for (uint32_t it = 0; it < iters; it++) fp2_mul28(x, x, y);
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < 14; i++) acc ^= x.c0.l[i] ^ x.c1.l[i];
  out[blockIdx.x * 64 + threadIdx.x] = acc;
}
__global__ void __launch_bounds__(64) k_chain2_eng(uint32_t *out, uint32_t iters, uint32_t seed) {
  gbls::fp2 x, y;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    y.c0.l[i] = (seed * 2654435761u + i * 97 + threadIdx.x) & 0x0fffffff;
    y.c1.l[i] = (seed * 40503u + i * 13 + threadIdx.x) & 0x0fffffff;
    x.c0.l[i] = (seed + i * 31 + blockIdx.x) & 0x0fffffff;
    x.c1.l[i] = (seed + i * 57 + blockIdx.x) & 0x0fffffff;
  }
  for (uint32_t it = 0; it < iters; it++) gbls::fp2_mul(x, x, y);
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) acc ^= x.c0.l[i] ^ x.c1.l[i];
  out[blockIdx.x * 64 + threadIdx.x] = acc;
}
__global__ void k_check2(const f28x2 *a, const f28x2 *b, f28x2 *r, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) fp2_mul28(r[i], a[i], b[i]);
}
template <bool ENGINE>
static void run2(uint32_t *sink, int waves, uint32_t iters) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int rep = 0; rep < 2; rep++) {
    hipEventRecord(e0);
    if (ENGINE)
      k_chain2_eng<<<waves, 64>>>(sink, iters, 3);
    else
      k_chain2_28<<<waves, 64>>>(sink, iters, 3);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
  }
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  printf("fp2_mul %-8s waves=%5d: %8.3f ms  %.3e Fp2-mul/s  per-lane latency %.3f us/mul\n",
         ENGINE ? "engine" : "radix28", waves, ms, (double)waves * 64 * iters / (ms * 1e-3),
         ms * 1e3 / iters);
}

template <int NACC>
__global__ void __launch_bounds__(64) k_chain(uint32_t *out, uint32_t iters, uint32_t seed) {
  f28 x, y;
#pragma unroll
  for (int i = 0; i < 14; i++) {
    y.l[i] = (seed * 2654435761u + i * 97 + threadIdx.x) & (i == 13 ? 0xffff : kM28);
    x.l[i] = (seed + i * 31 + blockIdx.x) & (i == 13 ? 0xffff : kM28);
  }
  for (uint32_t it = 0; it < iters; it++) mul28<NACC>(x, x, y);
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < 14; i++) acc ^= x.l[i];
  out[blockIdx.x * 64 + threadIdx.x] = acc;
}

__global__ void k_check(const f28 *a, const f28 *b, f28 *r, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) mul28<2>(r[i], a[i], b[i]);
}

template <int NACC>
static void run(uint32_t *sink, int waves, uint32_t iters) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  k_chain<NACC><<<waves, 64>>>(sink, iters, 1);
  hipEventRecord(e0);
  k_chain<NACC><<<waves, 64>>>(sink, iters, 3);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  double muls = (double)waves * 64 * iters;
  printf("radix28 nacc=%d waves=%5d (%.0f per SIMD): %8.3f ms  %.3e Fp-mul/s  per-lane latency %.3f us/mul\n",
         NACC, waves, waves / 1024.0, ms, muls / (ms * 1e-3), ms * 1e3 / iters);
}

int main(int argc, char **argv) {
  if (argc > 1 && !strcmp(argv[1], "check")) {
    const int n = 256;
    f28 ha[n], hb[n], hr[n];
    uint64_t s = 0x9e3779b97f4a7c15ull;
    for (int i = 0; i < n; i++)
      for (int j = 0; j < 14; j++) {
        s = s * 6364136223846793005ull + 1442695040888963407ull;
        // values < 2^381 < 2p (top limb < 2^17)
        ha[i].l[j] = (uint32_t)(s >> 36) & (j == 13 ? 0x1ffff : kM28);
        s = s * 6364136223846793005ull + 1442695040888963407ull;
        hb[i].l[j] = (uint32_t)(s >> 36) & (j == 13 ? 0x1ffff : kM28);
      }
    f28 *da, *db, *dr;
    hipMalloc(&da, sizeof ha);
    hipMalloc(&db, sizeof hb);
    hipMalloc(&dr, sizeof hr);
    hipMemcpy(da, ha, sizeof ha, hipMemcpyHostToDevice);
    hipMemcpy(db, hb, sizeof hb, hipMemcpyHostToDevice);
    k_check<<<(n + 63) / 64, 64>>>(da, db, dr, n);
    hipMemcpy(hr, dr, sizeof hr, hipMemcpyDeviceToHost);
    for (int i = 0; i < n; i++) {
      const f28 *v[3] = {&ha[i], &hb[i], &hr[i]};
      for (int w = 0; w < 3; w++) {
        for (int j = 0; j < 14; j++) printf("%s%x", j ? "," : "", v[w]->l[j]);
        printf(w < 2 ? " " : "\n");
      }
    }
    return 0;
  }
  if (argc > 1 && !strcmp(argv[1], "check2")) {
    const int n = 256;
    static f28x2 ha[n], hb[n], hr[n];
    uint64_t s = 0x243f6a8885a308d3ull;
    for (int i = 0; i < n; i++)
      for (int j = 0; j < 56; j++) {
        s = s * 6364136223846793005ull + 1442695040888963407ull;
        uint32_t v = (uint32_t)(s >> 36) & ((j % 14) == 13 ? 0x1ffff : kM28);
        f28 *dst = j < 14 ? &ha[i].c0 : j < 28 ? &ha[i].c1 : j < 42 ? &hb[i].c0 : &hb[i].c1;
        dst->l[j % 14] = v;
      }
    f28x2 *da, *db, *dr;
    hipMalloc(&da, sizeof ha);
    hipMalloc(&db, sizeof hb);
    hipMalloc(&dr, sizeof hr);
    hipMemcpy(da, ha, sizeof ha, hipMemcpyHostToDevice);
    hipMemcpy(db, hb, sizeof hb, hipMemcpyHostToDevice);
    k_check2<<<(n + 63) / 64, 64>>>(da, db, dr, n);
    hipMemcpy(hr, dr, sizeof hr, hipMemcpyDeviceToHost);
    for (int i = 0; i < n; i++) {
      const f28 *v[6] = {&ha[i].c0, &ha[i].c1, &hb[i].c0, &hb[i].c1, &hr[i].c0, &hr[i].c1};
      for (int w = 0; w < 6; w++) {
        for (int j = 0; j < 14; j++) printf("%s%x", j ? "," : "", v[w]->l[j]);
        printf(w < 5 ? " " : "\n");
      }
    }
    return 0;
  }
  uint32_t *sink;
  hipMalloc(&sink, 8192 * 64 * 4);
  run2<true>(sink, 1024, 1000);
  run2<false>(sink, 1024, 1000);
  run2<true>(sink, 2048, 1000);
  run2<false>(sink, 2048, 1000);
  const uint32_t it = 2000;
  run<1>(sink, 1024, it);
  run<2>(sink, 1024, it);
  run<4>(sink, 1024, it);
  run<2>(sink, 2048, it);
  run<2>(sink, 4096, it);
  run<1>(sink, 1024, it);
  printf("status %s\n", hipGetErrorString(hipDeviceSynchronize()));
  return 0;
}
