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

struct f28 {
  uint32_t l[14];
};

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
  uint32_t *sink;
  hipMalloc(&sink, 8192 * 64 * 4);
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
