#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include "/root/repo/grandine_amd/csrc/bls_constants.h"
using namespace gbls;
struct fpv { uint32_t l[12]; };
#define DI __device__ __forceinline__
DI void red(fpv &r, const uint32_t (&t)[12]) {
  uint32_t u[12]; uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) { uint64_t d = (uint64_t)t[i] - k::P[i] - br; u[i] = (uint32_t)d; br = (uint32_t)(d >> 63); }
  uint32_t msk = 0u - br;
#pragma unroll
  for (int i = 0; i < 12; i++) r.l[i] = (u[i] & ~msk) | (t[i] & msk);
}
DI void mul_single(fpv &r, const fpv &a, const fpv &b) {
  const uint32_t P0 = k::P[0];
  const uint32_t P1 = k::P[1];
  const uint32_t P2 = k::P[2];
  const uint32_t P3 = k::P[3];
  const uint32_t P4 = k::P[4];
  const uint32_t P5 = k::P[5];
  const uint32_t P6 = k::P[6];
  const uint32_t P7 = k::P[7];
  const uint32_t P8 = k::P[8];
  const uint32_t P9 = k::P[9];
  const uint32_t P10 = k::P[10];
  const uint32_t P11 = k::P[11];
  uint32_t m0, m1, m2, m3, m4, m5, m6, m7, m8, m9, m10, m11; uint32_t t[12];
  uint64_t acc0 = 0, acc1 = 0; uint32_t c20 = 0, c21 = 0; uint64_t sc0, sc1;
    asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
        : "+&v"(acc0), "+&v"(c20)
        : "v"(a.l[0]), "v"(b.l[0])
        : "vcc");
    m0 = (uint32_t)acc0 * k::PINV;
    asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
        : "+&v"(acc0), "+&v"(c20)
        : "v"(m0), "s"(P0)
        : "vcc");
    acc0 = (acc0 >> 32) | ((uint64_t)c20 << 32); c20 = 0;
    asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %4, %5, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %6, %7, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
        : "+&v"(acc0), "+&v"(c20)
        : "v"(a.l[0]), "v"(b.l[1]), "v"(a.l[1]), "v"(b.l[0]), "v"(m0), "s"(P1)
        : "vcc");
    m1 = (uint32_t)acc0 * k::PINV;
    asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
        : "+&v"(acc0), "+&v"(c20)
        : "v"(m1), "s"(P0)
        : "vcc");
    acc0 = (acc0 >> 32) | ((uint64_t)c20 << 32); c20 = 0;
    asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %4, %5, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %6, %7, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %8, %9, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %10, %11, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
        : "+&v"(acc0), "+&v"(c20)
        : "v"(a.l[0]), "v"(b.l[2]), "v"(a.l[1]), "v"(b.l[1]), "v"(a.l[2]), "v"(b.l[0]), "v"(m0), "s"(P2), "v"(m1), "s"(P1)
        : "vcc");
    m2 = (uint32_t)acc0 * k::PINV;
    asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
        : "+&v"(acc0), "+&v"(c20)
        : "v"(m2), "s"(P0)
        : "vcc");
    acc0 = (acc0 >> 32) | ((uint64_t)c20 << 32); c20 = 0;
    asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %4, %5, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %6, %7, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %8, %9, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %10, %11, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %12, %13, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %14, %15, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
        : "+&v"(acc0), "+&v"(c20)
        : "v"(a.l[0]), "v"(b.l[3]), "v"(a.l[1]), "v"(b.l[2]), "v"(a.l[2]), "v"(b.l[1]), "v"(a.l[3]), "v"(b.l[0]), "v"(m0), "s"(P3), "v"(m1), "s"(P2), "v"(m2), "s"(P1)
        : "vcc");
    m3 = (uint32_t)acc0 * k::PINV;
    asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
        : "+&v"(acc0), "+&v"(c20)
        : "v"(m3), "s"(P0)
        : "vcc");
    acc0 = (acc0 >> 32) | ((uint64_t)c20 << 32); c20 = 0;
    asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %4, %5, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %6, %7, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %8, %9, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %10, %11, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %12, %13, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %14, %15, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %16, %17, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %18, %19, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
        : "+&v"(acc0), "+&v"(c20)
        : "v"(a.l[0]), "v"(b.l[4]), "v"(a.l[1]), "v"(b.l[3]), "v"(a.l[2]), "v"(b.l[2]), "v"(a.l[3]), "v"(b.l[1]), "v"(a.l[4]), "v"(b.l[0]), "v"(m0), "s"(P4), "v"(m1), "s"(P3), "v"(m2), "s"(P2), "v"(m3), "s"(P1)
        : "vcc");
    m4 = (uint32_t)acc0 * k::PINV;
    asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
        : "+&v"(acc0), "+&v"(c20)
        : "v"(m4), "s"(P0)
        : "vcc");
    acc0 = (acc0 >> 32) | ((uint64_t)c20 << 32); c20 = 0;
    asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %4, %5, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %6, %7, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %8, %9, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %10, %11, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %12, %13, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %14, %15, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %16, %17, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %18, %19, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %20, %21, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %22, %23, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
        : "+&v"(acc0), "+&v"(c20)
        : "v"(a.l[0]), "v"(b.l[5]), "v"(a.l[1]), "v"(b.l[4]), "v"(a.l[2]), "v"(b.l[3]), "v"(a.l[3]), "v"(b.l[2]), "v"(a.l[4]), "v"(b.l[1]), "v"(a.l[5]), "v"(b.l[0]), "v"(m0), "s"(P5), "v"(m1), "s"(P4), "v"(m2), "s"(P3), "v"(m3), "s"(P2), "v"(m4), "s"(P1)
        : "vcc");
    m5 = (uint32_t)acc0 * k::PINV;
    asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
        : "+&v"(acc0), "+&v"(c20)
        : "v"(m5), "s"(P0)
        : "vcc");
    acc0 = (acc0 >> 32) | ((uint64_t)c20 << 32); c20 = 0;
    asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %4, %5, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %6, %7, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %8, %9, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %10, %11, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %12, %13, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %14, %15, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %16, %17, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %18, %19, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %20, %21, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %22, %23, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %24, %25, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %26, %27, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
        : "+&v"(acc0), "+&v"(c20)
        : "v"(a.l[0]), "v"(b.l[6]), "v"(a.l[1]), "v"(b.l[5]), "v"(a.l[2]), "v"(b.l[4]), "v"(a.l[3]), "v"(b.l[3]), "v"(a.l[4]), "v"(b.l[2]), "v"(a.l[5]), "v"(b.l[1]), "v"(a.l[6]), "v"(b.l[0]), "v"(m0), "s"(P6), "v"(m1), "s"(P5), "v"(m2), "s"(P4), "v"(m3), "s"(P3), "v"(m4), "s"(P2), "v"(m5), "s"(P1)
        : "vcc");
    m6 = (uint32_t)acc0 * k::PINV;
    asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
        : "+&v"(acc0), "+&v"(c20)
        : "v"(m6), "s"(P0)
        : "vcc");
    acc0 = (acc0 >> 32) | ((uint64_t)c20 << 32); c20 = 0;
    asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %4, %5, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %6, %7, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %8, %9, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %10, %11, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %12, %13, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %14, %15, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %16, %17, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %18, %19, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %20, %21, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %22, %23, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %24, %25, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %26, %27, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %28, %29, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %30, %31, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
        : "+&v"(acc0), "+&v"(c20)
        : "v"(a.l[0]), "v"(b.l[7]), "v"(a.l[1]), "v"(b.l[6]), "v"(a.l[2]), "v"(b.l[5]), "v"(a.l[3]), "v"(b.l[4]), "v"(a.l[4]), "v"(b.l[3]), "v"(a.l[5]), "v"(b.l[2]), "v"(a.l[6]), "v"(b.l[1]), "v"(a.l[7]), "v"(b.l[0]), "v"(m0), "s"(P7), "v"(m1), "s"(P6), "v"(m2), "s"(P5), "v"(m3), "s"(P4), "v"(m4), "s"(P3), "v"(m5), "s"(P2), "v"(m6), "s"(P1)
        : "vcc");
    m7 = (uint32_t)acc0 * k::PINV;
    asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
        : "+&v"(acc0), "+&v"(c20)
        : "v"(m7), "s"(P0)
        : "vcc");
    acc0 = (acc0 >> 32) | ((uint64_t)c20 << 32); c20 = 0;
    asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %4, %5, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %6, %7, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %8, %9, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %10, %11, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %12, %13, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %14, %15, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %16, %17, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %18, %19, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %20, %21, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %22, %23, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %24, %25, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %26, %27, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %28, %29, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %30, %31, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %32, %33, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %34, %35, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
        : "+&v"(acc0), "+&v"(c20)
        : "v"(a.l[0]), "v"(b.l[8]), "v"(a.l[1]), "v"(b.l[7]), "v"(a.l[2]), "v"(b.l[6]), "v"(a.l[3]), "v"(b.l[5]), "v"(a.l[4]), "v"(b.l[4]), "v"(a.l[5]), "v"(b.l[3]), "v"(a.l[6]), "v"(b.l[2]), "v"(a.l[7]), "v"(b.l[1]), "v"(a.l[8]), "v"(b.l[0]), "v"(m0), "s"(P8), "v"(m1), "s"(P7), "v"(m2), "s"(P6), "v"(m3), "s"(P5), "v"(m4), "s"(P4), "v"(m5), "s"(P3), "v"(m6), "s"(P2), "v"(m7), "s"(P1)
        : "vcc");
    m8 = (uint32_t)acc0 * k::PINV;
    asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
        : "+&v"(acc0), "+&v"(c20)
        : "v"(m8), "s"(P0)
        : "vcc");
    acc0 = (acc0 >> 32) | ((uint64_t)c20 << 32); c20 = 0;
    asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %4, %5, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %6, %7, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %8, %9, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %10, %11, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %12, %13, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %14, %15, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %16, %17, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %18, %19, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %20, %21, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %22, %23, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %24, %25, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %26, %27, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %28, %29, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %30, %31, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %32, %33, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %34, %35, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %36, %37, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %38, %39, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
        : "+&v"(acc0), "+&v"(c20)
        : "v"(a.l[0]), "v"(b.l[9]), "v"(a.l[1]), "v"(b.l[8]), "v"(a.l[2]), "v"(b.l[7]), "v"(a.l[3]), "v"(b.l[6]), "v"(a.l[4]), "v"(b.l[5]), "v"(a.l[5]), "v"(b.l[4]), "v"(a.l[6]), "v"(b.l[3]), "v"(a.l[7]), "v"(b.l[2]), "v"(a.l[8]), "v"(b.l[1]), "v"(a.l[9]), "v"(b.l[0]), "v"(m0), "s"(P9), "v"(m1), "s"(P8), "v"(m2), "s"(P7), "v"(m3), "s"(P6), "v"(m4), "s"(P5), "v"(m5), "s"(P4), "v"(m6), "s"(P3), "v"(m7), "s"(P2), "v"(m8), "s"(P1)
        : "vcc");
    m9 = (uint32_t)acc0 * k::PINV;
    asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
        : "+&v"(acc0), "+&v"(c20)
        : "v"(m9), "s"(P0)
        : "vcc");
    acc0 = (acc0 >> 32) | ((uint64_t)c20 << 32); c20 = 0;
    asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %4, %5, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %6, %7, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %8, %9, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %10, %11, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %12, %13, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %14, %15, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %16, %17, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %18, %19, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %20, %21, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %22, %23, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %24, %25, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %26, %27, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %28, %29, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %30, %31, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %32, %33, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %34, %35, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %36, %37, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %38, %39, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %40, %41, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %42, %43, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
        : "+&v"(acc0), "+&v"(c20)
        : "v"(a.l[0]), "v"(b.l[10]), "v"(a.l[1]), "v"(b.l[9]), "v"(a.l[2]), "v"(b.l[8]), "v"(a.l[3]), "v"(b.l[7]), "v"(a.l[4]), "v"(b.l[6]), "v"(a.l[5]), "v"(b.l[5]), "v"(a.l[6]), "v"(b.l[4]), "v"(a.l[7]), "v"(b.l[3]), "v"(a.l[8]), "v"(b.l[2]), "v"(a.l[9]), "v"(b.l[1]), "v"(a.l[10]), "v"(b.l[0]), "v"(m0), "s"(P10), "v"(m1), "s"(P9), "v"(m2), "s"(P8), "v"(m3), "s"(P7), "v"(m4), "s"(P6), "v"(m5), "s"(P5), "v"(m6), "s"(P4), "v"(m7), "s"(P3), "v"(m8), "s"(P2), "v"(m9), "s"(P1)
        : "vcc");
    m10 = (uint32_t)acc0 * k::PINV;
    asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
        : "+&v"(acc0), "+&v"(c20)
        : "v"(m10), "s"(P0)
        : "vcc");
    acc0 = (acc0 >> 32) | ((uint64_t)c20 << 32); c20 = 0;
    asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %4, %5, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %6, %7, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %8, %9, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %10, %11, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %12, %13, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %14, %15, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %16, %17, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %18, %19, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %20, %21, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %22, %23, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %24, %25, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %26, %27, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %28, %29, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %30, %31, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %32, %33, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %34, %35, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %36, %37, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %38, %39, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %40, %41, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %42, %43, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %44, %45, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %46, %47, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
        : "+&v"(acc0), "+&v"(c20)
        : "v"(a.l[0]), "v"(b.l[11]), "v"(a.l[1]), "v"(b.l[10]), "v"(a.l[2]), "v"(b.l[9]), "v"(a.l[3]), "v"(b.l[8]), "v"(a.l[4]), "v"(b.l[7]), "v"(a.l[5]), "v"(b.l[6]), "v"(a.l[6]), "v"(b.l[5]), "v"(a.l[7]), "v"(b.l[4]), "v"(a.l[8]), "v"(b.l[3]), "v"(a.l[9]), "v"(b.l[2]), "v"(a.l[10]), "v"(b.l[1]), "v"(a.l[11]), "v"(b.l[0]), "v"(m0), "s"(P11), "v"(m1), "s"(P10), "v"(m2), "s"(P9), "v"(m3), "s"(P8), "v"(m4), "s"(P7), "v"(m5), "s"(P6), "v"(m6), "s"(P5), "v"(m7), "s"(P4), "v"(m8), "s"(P3), "v"(m9), "s"(P2), "v"(m10), "s"(P1)
        : "vcc");
    m11 = (uint32_t)acc0 * k::PINV;
    asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
        : "+&v"(acc0), "+&v"(c20)
        : "v"(m11), "s"(P0)
        : "vcc");
    acc0 = (acc0 >> 32) | ((uint64_t)c20 << 32); c20 = 0;
    asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %4, %5, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %6, %7, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %8, %9, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %10, %11, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %12, %13, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %14, %15, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %16, %17, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %18, %19, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %20, %21, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %22, %23, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %24, %25, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %26, %27, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %28, %29, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %30, %31, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %32, %33, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %34, %35, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %36, %37, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %38, %39, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %40, %41, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %42, %43, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %44, %45, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
        : "+&v"(acc0), "+&v"(c20)
        : "v"(a.l[1]), "v"(b.l[11]), "v"(a.l[2]), "v"(b.l[10]), "v"(a.l[3]), "v"(b.l[9]), "v"(a.l[4]), "v"(b.l[8]), "v"(a.l[5]), "v"(b.l[7]), "v"(a.l[6]), "v"(b.l[6]), "v"(a.l[7]), "v"(b.l[5]), "v"(a.l[8]), "v"(b.l[4]), "v"(a.l[9]), "v"(b.l[3]), "v"(a.l[10]), "v"(b.l[2]), "v"(a.l[11]), "v"(b.l[1]), "v"(m1), "s"(P11), "v"(m2), "s"(P10), "v"(m3), "s"(P9), "v"(m4), "s"(P8), "v"(m5), "s"(P7), "v"(m6), "s"(P6), "v"(m7), "s"(P5), "v"(m8), "s"(P4), "v"(m9), "s"(P3), "v"(m10), "s"(P2), "v"(m11), "s"(P1)
        : "vcc");
    t[0] = (uint32_t)acc0;
    acc0 = (acc0 >> 32) | ((uint64_t)c20 << 32); c20 = 0;
    asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %4, %5, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %6, %7, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %8, %9, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %10, %11, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %12, %13, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %14, %15, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %16, %17, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %18, %19, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %20, %21, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %22, %23, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %24, %25, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %26, %27, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %28, %29, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %30, %31, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %32, %33, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %34, %35, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %36, %37, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %38, %39, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %40, %41, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
        : "+&v"(acc0), "+&v"(c20)
        : "v"(a.l[2]), "v"(b.l[11]), "v"(a.l[3]), "v"(b.l[10]), "v"(a.l[4]), "v"(b.l[9]), "v"(a.l[5]), "v"(b.l[8]), "v"(a.l[6]), "v"(b.l[7]), "v"(a.l[7]), "v"(b.l[6]), "v"(a.l[8]), "v"(b.l[5]), "v"(a.l[9]), "v"(b.l[4]), "v"(a.l[10]), "v"(b.l[3]), "v"(a.l[11]), "v"(b.l[2]), "v"(m2), "s"(P11), "v"(m3), "s"(P10), "v"(m4), "s"(P9), "v"(m5), "s"(P8), "v"(m6), "s"(P7), "v"(m7), "s"(P6), "v"(m8), "s"(P5), "v"(m9), "s"(P4), "v"(m10), "s"(P3), "v"(m11), "s"(P2)
        : "vcc");
    t[1] = (uint32_t)acc0;
    acc0 = (acc0 >> 32) | ((uint64_t)c20 << 32); c20 = 0;
    asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %4, %5, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %6, %7, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %8, %9, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %10, %11, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %12, %13, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %14, %15, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %16, %17, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %18, %19, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %20, %21, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %22, %23, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %24, %25, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %26, %27, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %28, %29, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %30, %31, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %32, %33, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %34, %35, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %36, %37, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
        : "+&v"(acc0), "+&v"(c20)
        : "v"(a.l[3]), "v"(b.l[11]), "v"(a.l[4]), "v"(b.l[10]), "v"(a.l[5]), "v"(b.l[9]), "v"(a.l[6]), "v"(b.l[8]), "v"(a.l[7]), "v"(b.l[7]), "v"(a.l[8]), "v"(b.l[6]), "v"(a.l[9]), "v"(b.l[5]), "v"(a.l[10]), "v"(b.l[4]), "v"(a.l[11]), "v"(b.l[3]), "v"(m3), "s"(P11), "v"(m4), "s"(P10), "v"(m5), "s"(P9), "v"(m6), "s"(P8), "v"(m7), "s"(P7), "v"(m8), "s"(P6), "v"(m9), "s"(P5), "v"(m10), "s"(P4), "v"(m11), "s"(P3)
        : "vcc");
    t[2] = (uint32_t)acc0;
    acc0 = (acc0 >> 32) | ((uint64_t)c20 << 32); c20 = 0;
    asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %4, %5, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %6, %7, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %8, %9, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %10, %11, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %12, %13, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %14, %15, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %16, %17, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %18, %19, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %20, %21, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %22, %23, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %24, %25, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %26, %27, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %28, %29, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %30, %31, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %32, %33, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
        : "+&v"(acc0), "+&v"(c20)
        : "v"(a.l[4]), "v"(b.l[11]), "v"(a.l[5]), "v"(b.l[10]), "v"(a.l[6]), "v"(b.l[9]), "v"(a.l[7]), "v"(b.l[8]), "v"(a.l[8]), "v"(b.l[7]), "v"(a.l[9]), "v"(b.l[6]), "v"(a.l[10]), "v"(b.l[5]), "v"(a.l[11]), "v"(b.l[4]), "v"(m4), "s"(P11), "v"(m5), "s"(P10), "v"(m6), "s"(P9), "v"(m7), "s"(P8), "v"(m8), "s"(P7), "v"(m9), "s"(P6), "v"(m10), "s"(P5), "v"(m11), "s"(P4)
        : "vcc");
    t[3] = (uint32_t)acc0;
    acc0 = (acc0 >> 32) | ((uint64_t)c20 << 32); c20 = 0;
    asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %4, %5, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %6, %7, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %8, %9, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %10, %11, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %12, %13, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %14, %15, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %16, %17, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %18, %19, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %20, %21, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %22, %23, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %24, %25, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %26, %27, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %28, %29, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
        : "+&v"(acc0), "+&v"(c20)
        : "v"(a.l[5]), "v"(b.l[11]), "v"(a.l[6]), "v"(b.l[10]), "v"(a.l[7]), "v"(b.l[9]), "v"(a.l[8]), "v"(b.l[8]), "v"(a.l[9]), "v"(b.l[7]), "v"(a.l[10]), "v"(b.l[6]), "v"(a.l[11]), "v"(b.l[5]), "v"(m5), "s"(P11), "v"(m6), "s"(P10), "v"(m7), "s"(P9), "v"(m8), "s"(P8), "v"(m9), "s"(P7), "v"(m10), "s"(P6), "v"(m11), "s"(P5)
        : "vcc");
    t[4] = (uint32_t)acc0;
    acc0 = (acc0 >> 32) | ((uint64_t)c20 << 32); c20 = 0;
    asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %4, %5, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %6, %7, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %8, %9, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %10, %11, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %12, %13, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %14, %15, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %16, %17, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %18, %19, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %20, %21, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %22, %23, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %24, %25, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
        : "+&v"(acc0), "+&v"(c20)
        : "v"(a.l[6]), "v"(b.l[11]), "v"(a.l[7]), "v"(b.l[10]), "v"(a.l[8]), "v"(b.l[9]), "v"(a.l[9]), "v"(b.l[8]), "v"(a.l[10]), "v"(b.l[7]), "v"(a.l[11]), "v"(b.l[6]), "v"(m6), "s"(P11), "v"(m7), "s"(P10), "v"(m8), "s"(P9), "v"(m9), "s"(P8), "v"(m10), "s"(P7), "v"(m11), "s"(P6)
        : "vcc");
    t[5] = (uint32_t)acc0;
    acc0 = (acc0 >> 32) | ((uint64_t)c20 << 32); c20 = 0;
    asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %4, %5, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %6, %7, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %8, %9, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %10, %11, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %12, %13, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %14, %15, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %16, %17, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %18, %19, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %20, %21, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
        : "+&v"(acc0), "+&v"(c20)
        : "v"(a.l[7]), "v"(b.l[11]), "v"(a.l[8]), "v"(b.l[10]), "v"(a.l[9]), "v"(b.l[9]), "v"(a.l[10]), "v"(b.l[8]), "v"(a.l[11]), "v"(b.l[7]), "v"(m7), "s"(P11), "v"(m8), "s"(P10), "v"(m9), "s"(P9), "v"(m10), "s"(P8), "v"(m11), "s"(P7)
        : "vcc");
    t[6] = (uint32_t)acc0;
    acc0 = (acc0 >> 32) | ((uint64_t)c20 << 32); c20 = 0;
    asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %4, %5, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %6, %7, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %8, %9, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %10, %11, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %12, %13, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %14, %15, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %16, %17, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
        : "+&v"(acc0), "+&v"(c20)
        : "v"(a.l[8]), "v"(b.l[11]), "v"(a.l[9]), "v"(b.l[10]), "v"(a.l[10]), "v"(b.l[9]), "v"(a.l[11]), "v"(b.l[8]), "v"(m8), "s"(P11), "v"(m9), "s"(P10), "v"(m10), "s"(P9), "v"(m11), "s"(P8)
        : "vcc");
    t[7] = (uint32_t)acc0;
    acc0 = (acc0 >> 32) | ((uint64_t)c20 << 32); c20 = 0;
    asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %4, %5, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %6, %7, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %8, %9, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %10, %11, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %12, %13, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
        : "+&v"(acc0), "+&v"(c20)
        : "v"(a.l[9]), "v"(b.l[11]), "v"(a.l[10]), "v"(b.l[10]), "v"(a.l[11]), "v"(b.l[9]), "v"(m9), "s"(P11), "v"(m10), "s"(P10), "v"(m11), "s"(P9)
        : "vcc");
    t[8] = (uint32_t)acc0;
    acc0 = (acc0 >> 32) | ((uint64_t)c20 << 32); c20 = 0;
    asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %4, %5, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %6, %7, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %8, %9, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
        : "+&v"(acc0), "+&v"(c20)
        : "v"(a.l[10]), "v"(b.l[11]), "v"(a.l[11]), "v"(b.l[10]), "v"(m10), "s"(P11), "v"(m11), "s"(P10)
        : "vcc");
    t[9] = (uint32_t)acc0;
    acc0 = (acc0 >> 32) | ((uint64_t)c20 << 32); c20 = 0;
    asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_mad_u64_u32 %0, vcc, %4, %5, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
        : "+&v"(acc0), "+&v"(c20)
        : "v"(a.l[11]), "v"(b.l[11]), "v"(m11), "s"(P11)
        : "vcc");
    t[10] = (uint32_t)acc0;
    acc0 = (acc0 >> 32) | ((uint64_t)c20 << 32); c20 = 0;
  t[11] = (uint32_t)acc0;
  red(r, t);
}
DI void mul_dual(fpv &r, const fpv &a, const fpv &b) {
  const uint32_t P0 = k::P[0];
  const uint32_t P1 = k::P[1];
  const uint32_t P2 = k::P[2];
  const uint32_t P3 = k::P[3];
  const uint32_t P4 = k::P[4];
  const uint32_t P5 = k::P[5];
  const uint32_t P6 = k::P[6];
  const uint32_t P7 = k::P[7];
  const uint32_t P8 = k::P[8];
  const uint32_t P9 = k::P[9];
  const uint32_t P10 = k::P[10];
  const uint32_t P11 = k::P[11];
  uint32_t m0, m1, m2, m3, m4, m5, m6, m7, m8, m9, m10, m11; uint32_t t[12];
  uint64_t acc0 = 0, acc1 = 0; uint32_t c20 = 0, c21 = 0; uint64_t sc0, sc1;
    asm volatile("v_mad_u64_u32 %0, %4, %6, %7, %0\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4"
        : "+&v"(acc0), "+&v"(acc1), "+&v"(c20), "+&v"(c21), "=&s"(sc0), "=&s"(sc1)
        : "v"(a.l[0]), "v"(b.l[0])
        : "vcc");
    { uint64_t s = acc0 + acc1; c20 = c20 + c21 + (uint32_t)(s < acc0); acc0 = s; acc1 = 0; c21 = 0; }
    m0 = (uint32_t)acc0 * k::PINV;
    asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
        : "+&v"(acc0), "+&v"(c20)
        : "v"(m0), "s"(P0)
        : "vcc");
    acc0 = (acc0 >> 32) | ((uint64_t)c20 << 32); c20 = 0;
    asm volatile("v_mad_u64_u32 %0, %4, %6, %7, %0\n\tv_mad_u64_u32 %1, %5, %8, %9, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %10, %11, %0\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4"
        : "+&v"(acc0), "+&v"(acc1), "+&v"(c20), "+&v"(c21), "=&s"(sc0), "=&s"(sc1)
        : "v"(a.l[0]), "v"(b.l[1]), "v"(a.l[1]), "v"(b.l[0]), "v"(m0), "s"(P1)
        : "vcc");
    { uint64_t s = acc0 + acc1; c20 = c20 + c21 + (uint32_t)(s < acc0); acc0 = s; acc1 = 0; c21 = 0; }
    m1 = (uint32_t)acc0 * k::PINV;
    asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
        : "+&v"(acc0), "+&v"(c20)
        : "v"(m1), "s"(P0)
        : "vcc");
    acc0 = (acc0 >> 32) | ((uint64_t)c20 << 32); c20 = 0;
    asm volatile("v_mad_u64_u32 %0, %4, %6, %7, %0\n\tv_mad_u64_u32 %1, %5, %8, %9, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %10, %11, %0\n\tv_mad_u64_u32 %1, %5, %12, %13, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %14, %15, %0\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4"
        : "+&v"(acc0), "+&v"(acc1), "+&v"(c20), "+&v"(c21), "=&s"(sc0), "=&s"(sc1)
        : "v"(a.l[0]), "v"(b.l[2]), "v"(a.l[1]), "v"(b.l[1]), "v"(a.l[2]), "v"(b.l[0]), "v"(m0), "s"(P2), "v"(m1), "s"(P1)
        : "vcc");
    { uint64_t s = acc0 + acc1; c20 = c20 + c21 + (uint32_t)(s < acc0); acc0 = s; acc1 = 0; c21 = 0; }
    m2 = (uint32_t)acc0 * k::PINV;
    asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
        : "+&v"(acc0), "+&v"(c20)
        : "v"(m2), "s"(P0)
        : "vcc");
    acc0 = (acc0 >> 32) | ((uint64_t)c20 << 32); c20 = 0;
    asm volatile("v_mad_u64_u32 %0, %4, %6, %7, %0\n\tv_mad_u64_u32 %1, %5, %8, %9, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %10, %11, %0\n\tv_mad_u64_u32 %1, %5, %12, %13, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %14, %15, %0\n\tv_mad_u64_u32 %1, %5, %16, %17, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %18, %19, %0\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4"
        : "+&v"(acc0), "+&v"(acc1), "+&v"(c20), "+&v"(c21), "=&s"(sc0), "=&s"(sc1)
        : "v"(a.l[0]), "v"(b.l[3]), "v"(a.l[1]), "v"(b.l[2]), "v"(a.l[2]), "v"(b.l[1]), "v"(a.l[3]), "v"(b.l[0]), "v"(m0), "s"(P3), "v"(m1), "s"(P2), "v"(m2), "s"(P1)
        : "vcc");
    { uint64_t s = acc0 + acc1; c20 = c20 + c21 + (uint32_t)(s < acc0); acc0 = s; acc1 = 0; c21 = 0; }
    m3 = (uint32_t)acc0 * k::PINV;
    asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
        : "+&v"(acc0), "+&v"(c20)
        : "v"(m3), "s"(P0)
        : "vcc");
    acc0 = (acc0 >> 32) | ((uint64_t)c20 << 32); c20 = 0;
    asm volatile("v_mad_u64_u32 %0, %4, %6, %7, %0\n\tv_mad_u64_u32 %1, %5, %8, %9, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %10, %11, %0\n\tv_mad_u64_u32 %1, %5, %12, %13, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %14, %15, %0\n\tv_mad_u64_u32 %1, %5, %16, %17, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %18, %19, %0\n\tv_mad_u64_u32 %1, %5, %20, %21, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %22, %23, %0\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4"
        : "+&v"(acc0), "+&v"(acc1), "+&v"(c20), "+&v"(c21), "=&s"(sc0), "=&s"(sc1)
        : "v"(a.l[0]), "v"(b.l[4]), "v"(a.l[1]), "v"(b.l[3]), "v"(a.l[2]), "v"(b.l[2]), "v"(a.l[3]), "v"(b.l[1]), "v"(a.l[4]), "v"(b.l[0]), "v"(m0), "s"(P4), "v"(m1), "s"(P3), "v"(m2), "s"(P2), "v"(m3), "s"(P1)
        : "vcc");
    { uint64_t s = acc0 + acc1; c20 = c20 + c21 + (uint32_t)(s < acc0); acc0 = s; acc1 = 0; c21 = 0; }
    m4 = (uint32_t)acc0 * k::PINV;
    asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
        : "+&v"(acc0), "+&v"(c20)
        : "v"(m4), "s"(P0)
        : "vcc");
    acc0 = (acc0 >> 32) | ((uint64_t)c20 << 32); c20 = 0;
    asm volatile("v_mad_u64_u32 %0, %4, %6, %7, %0\n\tv_mad_u64_u32 %1, %5, %8, %9, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %10, %11, %0\n\tv_mad_u64_u32 %1, %5, %12, %13, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %14, %15, %0\n\tv_mad_u64_u32 %1, %5, %16, %17, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %18, %19, %0\n\tv_mad_u64_u32 %1, %5, %20, %21, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %22, %23, %0\n\tv_mad_u64_u32 %1, %5, %24, %25, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %26, %27, %0\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4"
        : "+&v"(acc0), "+&v"(acc1), "+&v"(c20), "+&v"(c21), "=&s"(sc0), "=&s"(sc1)
        : "v"(a.l[0]), "v"(b.l[5]), "v"(a.l[1]), "v"(b.l[4]), "v"(a.l[2]), "v"(b.l[3]), "v"(a.l[3]), "v"(b.l[2]), "v"(a.l[4]), "v"(b.l[1]), "v"(a.l[5]), "v"(b.l[0]), "v"(m0), "s"(P5), "v"(m1), "s"(P4), "v"(m2), "s"(P3), "v"(m3), "s"(P2), "v"(m4), "s"(P1)
        : "vcc");
    { uint64_t s = acc0 + acc1; c20 = c20 + c21 + (uint32_t)(s < acc0); acc0 = s; acc1 = 0; c21 = 0; }
    m5 = (uint32_t)acc0 * k::PINV;
    asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
        : "+&v"(acc0), "+&v"(c20)
        : "v"(m5), "s"(P0)
        : "vcc");
    acc0 = (acc0 >> 32) | ((uint64_t)c20 << 32); c20 = 0;
    asm volatile("v_mad_u64_u32 %0, %4, %6, %7, %0\n\tv_mad_u64_u32 %1, %5, %8, %9, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %10, %11, %0\n\tv_mad_u64_u32 %1, %5, %12, %13, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %14, %15, %0\n\tv_mad_u64_u32 %1, %5, %16, %17, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %18, %19, %0\n\tv_mad_u64_u32 %1, %5, %20, %21, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %22, %23, %0\n\tv_mad_u64_u32 %1, %5, %24, %25, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %26, %27, %0\n\tv_mad_u64_u32 %1, %5, %28, %29, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %30, %31, %0\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4"
        : "+&v"(acc0), "+&v"(acc1), "+&v"(c20), "+&v"(c21), "=&s"(sc0), "=&s"(sc1)
        : "v"(a.l[0]), "v"(b.l[6]), "v"(a.l[1]), "v"(b.l[5]), "v"(a.l[2]), "v"(b.l[4]), "v"(a.l[3]), "v"(b.l[3]), "v"(a.l[4]), "v"(b.l[2]), "v"(a.l[5]), "v"(b.l[1]), "v"(a.l[6]), "v"(b.l[0]), "v"(m0), "s"(P6), "v"(m1), "s"(P5), "v"(m2), "s"(P4), "v"(m3), "s"(P3), "v"(m4), "s"(P2), "v"(m5), "s"(P1)
        : "vcc");
    { uint64_t s = acc0 + acc1; c20 = c20 + c21 + (uint32_t)(s < acc0); acc0 = s; acc1 = 0; c21 = 0; }
    m6 = (uint32_t)acc0 * k::PINV;
    asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
        : "+&v"(acc0), "+&v"(c20)
        : "v"(m6), "s"(P0)
        : "vcc");
    acc0 = (acc0 >> 32) | ((uint64_t)c20 << 32); c20 = 0;
    asm volatile("v_mad_u64_u32 %0, %4, %6, %7, %0\n\tv_mad_u64_u32 %1, %5, %8, %9, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %10, %11, %0\n\tv_mad_u64_u32 %1, %5, %12, %13, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %14, %15, %0\n\tv_mad_u64_u32 %1, %5, %16, %17, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %18, %19, %0\n\tv_mad_u64_u32 %1, %5, %20, %21, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %22, %23, %0\n\tv_mad_u64_u32 %1, %5, %24, %25, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %26, %27, %0\n\tv_mad_u64_u32 %1, %5, %28, %29, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %30, %31, %0\n\tv_mad_u64_u32 %1, %5, %32, %33, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %34, %35, %0\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4"
        : "+&v"(acc0), "+&v"(acc1), "+&v"(c20), "+&v"(c21), "=&s"(sc0), "=&s"(sc1)
        : "v"(a.l[0]), "v"(b.l[7]), "v"(a.l[1]), "v"(b.l[6]), "v"(a.l[2]), "v"(b.l[5]), "v"(a.l[3]), "v"(b.l[4]), "v"(a.l[4]), "v"(b.l[3]), "v"(a.l[5]), "v"(b.l[2]), "v"(a.l[6]), "v"(b.l[1]), "v"(a.l[7]), "v"(b.l[0]), "v"(m0), "s"(P7), "v"(m1), "s"(P6), "v"(m2), "s"(P5), "v"(m3), "s"(P4), "v"(m4), "s"(P3), "v"(m5), "s"(P2), "v"(m6), "s"(P1)
        : "vcc");
    { uint64_t s = acc0 + acc1; c20 = c20 + c21 + (uint32_t)(s < acc0); acc0 = s; acc1 = 0; c21 = 0; }
    m7 = (uint32_t)acc0 * k::PINV;
    asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
        : "+&v"(acc0), "+&v"(c20)
        : "v"(m7), "s"(P0)
        : "vcc");
    acc0 = (acc0 >> 32) | ((uint64_t)c20 << 32); c20 = 0;
    asm volatile("v_mad_u64_u32 %0, %4, %6, %7, %0\n\tv_mad_u64_u32 %1, %5, %8, %9, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %10, %11, %0\n\tv_mad_u64_u32 %1, %5, %12, %13, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %14, %15, %0\n\tv_mad_u64_u32 %1, %5, %16, %17, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %18, %19, %0\n\tv_mad_u64_u32 %1, %5, %20, %21, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %22, %23, %0\n\tv_mad_u64_u32 %1, %5, %24, %25, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %26, %27, %0\n\tv_mad_u64_u32 %1, %5, %28, %29, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %30, %31, %0\n\tv_mad_u64_u32 %1, %5, %32, %33, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %34, %35, %0\n\tv_mad_u64_u32 %1, %5, %36, %37, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %38, %39, %0\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4"
        : "+&v"(acc0), "+&v"(acc1), "+&v"(c20), "+&v"(c21), "=&s"(sc0), "=&s"(sc1)
        : "v"(a.l[0]), "v"(b.l[8]), "v"(a.l[1]), "v"(b.l[7]), "v"(a.l[2]), "v"(b.l[6]), "v"(a.l[3]), "v"(b.l[5]), "v"(a.l[4]), "v"(b.l[4]), "v"(a.l[5]), "v"(b.l[3]), "v"(a.l[6]), "v"(b.l[2]), "v"(a.l[7]), "v"(b.l[1]), "v"(a.l[8]), "v"(b.l[0]), "v"(m0), "s"(P8), "v"(m1), "s"(P7), "v"(m2), "s"(P6), "v"(m3), "s"(P5), "v"(m4), "s"(P4), "v"(m5), "s"(P3), "v"(m6), "s"(P2), "v"(m7), "s"(P1)
        : "vcc");
    { uint64_t s = acc0 + acc1; c20 = c20 + c21 + (uint32_t)(s < acc0); acc0 = s; acc1 = 0; c21 = 0; }
    m8 = (uint32_t)acc0 * k::PINV;
    asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
        : "+&v"(acc0), "+&v"(c20)
        : "v"(m8), "s"(P0)
        : "vcc");
    acc0 = (acc0 >> 32) | ((uint64_t)c20 << 32); c20 = 0;
    asm volatile("v_mad_u64_u32 %0, %4, %6, %7, %0\n\tv_mad_u64_u32 %1, %5, %8, %9, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %10, %11, %0\n\tv_mad_u64_u32 %1, %5, %12, %13, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %14, %15, %0\n\tv_mad_u64_u32 %1, %5, %16, %17, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %18, %19, %0\n\tv_mad_u64_u32 %1, %5, %20, %21, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %22, %23, %0\n\tv_mad_u64_u32 %1, %5, %24, %25, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %26, %27, %0\n\tv_mad_u64_u32 %1, %5, %28, %29, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %30, %31, %0\n\tv_mad_u64_u32 %1, %5, %32, %33, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %34, %35, %0\n\tv_mad_u64_u32 %1, %5, %36, %37, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %38, %39, %0\n\tv_mad_u64_u32 %1, %5, %40, %41, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %42, %43, %0\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4"
        : "+&v"(acc0), "+&v"(acc1), "+&v"(c20), "+&v"(c21), "=&s"(sc0), "=&s"(sc1)
        : "v"(a.l[0]), "v"(b.l[9]), "v"(a.l[1]), "v"(b.l[8]), "v"(a.l[2]), "v"(b.l[7]), "v"(a.l[3]), "v"(b.l[6]), "v"(a.l[4]), "v"(b.l[5]), "v"(a.l[5]), "v"(b.l[4]), "v"(a.l[6]), "v"(b.l[3]), "v"(a.l[7]), "v"(b.l[2]), "v"(a.l[8]), "v"(b.l[1]), "v"(a.l[9]), "v"(b.l[0]), "v"(m0), "s"(P9), "v"(m1), "s"(P8), "v"(m2), "s"(P7), "v"(m3), "s"(P6), "v"(m4), "s"(P5), "v"(m5), "s"(P4), "v"(m6), "s"(P3), "v"(m7), "s"(P2), "v"(m8), "s"(P1)
        : "vcc");
    { uint64_t s = acc0 + acc1; c20 = c20 + c21 + (uint32_t)(s < acc0); acc0 = s; acc1 = 0; c21 = 0; }
    m9 = (uint32_t)acc0 * k::PINV;
    asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
        : "+&v"(acc0), "+&v"(c20)
        : "v"(m9), "s"(P0)
        : "vcc");
    acc0 = (acc0 >> 32) | ((uint64_t)c20 << 32); c20 = 0;
    asm volatile("v_mad_u64_u32 %0, %4, %6, %7, %0\n\tv_mad_u64_u32 %1, %5, %8, %9, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %10, %11, %0\n\tv_mad_u64_u32 %1, %5, %12, %13, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %14, %15, %0\n\tv_mad_u64_u32 %1, %5, %16, %17, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %18, %19, %0\n\tv_mad_u64_u32 %1, %5, %20, %21, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %22, %23, %0\n\tv_mad_u64_u32 %1, %5, %24, %25, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %26, %27, %0\n\tv_mad_u64_u32 %1, %5, %28, %29, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %30, %31, %0\n\tv_mad_u64_u32 %1, %5, %32, %33, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %34, %35, %0\n\tv_mad_u64_u32 %1, %5, %36, %37, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %38, %39, %0\n\tv_mad_u64_u32 %1, %5, %40, %41, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %42, %43, %0\n\tv_mad_u64_u32 %1, %5, %44, %45, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %46, %47, %0\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4"
        : "+&v"(acc0), "+&v"(acc1), "+&v"(c20), "+&v"(c21), "=&s"(sc0), "=&s"(sc1)
        : "v"(a.l[0]), "v"(b.l[10]), "v"(a.l[1]), "v"(b.l[9]), "v"(a.l[2]), "v"(b.l[8]), "v"(a.l[3]), "v"(b.l[7]), "v"(a.l[4]), "v"(b.l[6]), "v"(a.l[5]), "v"(b.l[5]), "v"(a.l[6]), "v"(b.l[4]), "v"(a.l[7]), "v"(b.l[3]), "v"(a.l[8]), "v"(b.l[2]), "v"(a.l[9]), "v"(b.l[1]), "v"(a.l[10]), "v"(b.l[0]), "v"(m0), "s"(P10), "v"(m1), "s"(P9), "v"(m2), "s"(P8), "v"(m3), "s"(P7), "v"(m4), "s"(P6), "v"(m5), "s"(P5), "v"(m6), "s"(P4), "v"(m7), "s"(P3), "v"(m8), "s"(P2), "v"(m9), "s"(P1)
        : "vcc");
    { uint64_t s = acc0 + acc1; c20 = c20 + c21 + (uint32_t)(s < acc0); acc0 = s; acc1 = 0; c21 = 0; }
    m10 = (uint32_t)acc0 * k::PINV;
    asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
        : "+&v"(acc0), "+&v"(c20)
        : "v"(m10), "s"(P0)
        : "vcc");
    acc0 = (acc0 >> 32) | ((uint64_t)c20 << 32); c20 = 0;
    asm volatile("v_mad_u64_u32 %0, %4, %6, %7, %0\n\tv_mad_u64_u32 %1, %5, %8, %9, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %10, %11, %0\n\tv_mad_u64_u32 %1, %5, %12, %13, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %14, %15, %0\n\tv_mad_u64_u32 %1, %5, %16, %17, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %18, %19, %0\n\tv_mad_u64_u32 %1, %5, %20, %21, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %22, %23, %0\n\tv_mad_u64_u32 %1, %5, %24, %25, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %26, %27, %0\n\tv_mad_u64_u32 %1, %5, %28, %29, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %30, %31, %0\n\tv_mad_u64_u32 %1, %5, %32, %33, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %34, %35, %0\n\tv_mad_u64_u32 %1, %5, %36, %37, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %38, %39, %0\n\tv_mad_u64_u32 %1, %5, %40, %41, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %42, %43, %0\n\tv_mad_u64_u32 %1, %5, %44, %45, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %46, %47, %0\n\tv_mad_u64_u32 %1, %5, %48, %49, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %50, %51, %0\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4"
        : "+&v"(acc0), "+&v"(acc1), "+&v"(c20), "+&v"(c21), "=&s"(sc0), "=&s"(sc1)
        : "v"(a.l[0]), "v"(b.l[11]), "v"(a.l[1]), "v"(b.l[10]), "v"(a.l[2]), "v"(b.l[9]), "v"(a.l[3]), "v"(b.l[8]), "v"(a.l[4]), "v"(b.l[7]), "v"(a.l[5]), "v"(b.l[6]), "v"(a.l[6]), "v"(b.l[5]), "v"(a.l[7]), "v"(b.l[4]), "v"(a.l[8]), "v"(b.l[3]), "v"(a.l[9]), "v"(b.l[2]), "v"(a.l[10]), "v"(b.l[1]), "v"(a.l[11]), "v"(b.l[0]), "v"(m0), "s"(P11), "v"(m1), "s"(P10), "v"(m2), "s"(P9), "v"(m3), "s"(P8), "v"(m4), "s"(P7), "v"(m5), "s"(P6), "v"(m6), "s"(P5), "v"(m7), "s"(P4), "v"(m8), "s"(P3), "v"(m9), "s"(P2), "v"(m10), "s"(P1)
        : "vcc");
    { uint64_t s = acc0 + acc1; c20 = c20 + c21 + (uint32_t)(s < acc0); acc0 = s; acc1 = 0; c21 = 0; }
    m11 = (uint32_t)acc0 * k::PINV;
    asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
        : "+&v"(acc0), "+&v"(c20)
        : "v"(m11), "s"(P0)
        : "vcc");
    acc0 = (acc0 >> 32) | ((uint64_t)c20 << 32); c20 = 0;
    asm volatile("v_mad_u64_u32 %0, %4, %6, %7, %0\n\tv_mad_u64_u32 %1, %5, %8, %9, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %10, %11, %0\n\tv_mad_u64_u32 %1, %5, %12, %13, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %14, %15, %0\n\tv_mad_u64_u32 %1, %5, %16, %17, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %18, %19, %0\n\tv_mad_u64_u32 %1, %5, %20, %21, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %22, %23, %0\n\tv_mad_u64_u32 %1, %5, %24, %25, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %26, %27, %0\n\tv_mad_u64_u32 %1, %5, %28, %29, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %30, %31, %0\n\tv_mad_u64_u32 %1, %5, %32, %33, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %34, %35, %0\n\tv_mad_u64_u32 %1, %5, %36, %37, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %38, %39, %0\n\tv_mad_u64_u32 %1, %5, %40, %41, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %42, %43, %0\n\tv_mad_u64_u32 %1, %5, %44, %45, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %46, %47, %0\n\tv_mad_u64_u32 %1, %5, %48, %49, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5"
        : "+&v"(acc0), "+&v"(acc1), "+&v"(c20), "+&v"(c21), "=&s"(sc0), "=&s"(sc1)
        : "v"(a.l[1]), "v"(b.l[11]), "v"(a.l[2]), "v"(b.l[10]), "v"(a.l[3]), "v"(b.l[9]), "v"(a.l[4]), "v"(b.l[8]), "v"(a.l[5]), "v"(b.l[7]), "v"(a.l[6]), "v"(b.l[6]), "v"(a.l[7]), "v"(b.l[5]), "v"(a.l[8]), "v"(b.l[4]), "v"(a.l[9]), "v"(b.l[3]), "v"(a.l[10]), "v"(b.l[2]), "v"(a.l[11]), "v"(b.l[1]), "v"(m1), "s"(P11), "v"(m2), "s"(P10), "v"(m3), "s"(P9), "v"(m4), "s"(P8), "v"(m5), "s"(P7), "v"(m6), "s"(P6), "v"(m7), "s"(P5), "v"(m8), "s"(P4), "v"(m9), "s"(P3), "v"(m10), "s"(P2), "v"(m11), "s"(P1)
        : "vcc");
    { uint64_t s = acc0 + acc1; c20 = c20 + c21 + (uint32_t)(s < acc0); acc0 = s; acc1 = 0; c21 = 0; }
    t[0] = (uint32_t)acc0;
    acc0 = (acc0 >> 32) | ((uint64_t)c20 << 32); c20 = 0;
    asm volatile("v_mad_u64_u32 %0, %4, %6, %7, %0\n\tv_mad_u64_u32 %1, %5, %8, %9, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %10, %11, %0\n\tv_mad_u64_u32 %1, %5, %12, %13, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %14, %15, %0\n\tv_mad_u64_u32 %1, %5, %16, %17, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %18, %19, %0\n\tv_mad_u64_u32 %1, %5, %20, %21, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %22, %23, %0\n\tv_mad_u64_u32 %1, %5, %24, %25, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %26, %27, %0\n\tv_mad_u64_u32 %1, %5, %28, %29, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %30, %31, %0\n\tv_mad_u64_u32 %1, %5, %32, %33, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %34, %35, %0\n\tv_mad_u64_u32 %1, %5, %36, %37, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %38, %39, %0\n\tv_mad_u64_u32 %1, %5, %40, %41, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %42, %43, %0\n\tv_mad_u64_u32 %1, %5, %44, %45, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5"
        : "+&v"(acc0), "+&v"(acc1), "+&v"(c20), "+&v"(c21), "=&s"(sc0), "=&s"(sc1)
        : "v"(a.l[2]), "v"(b.l[11]), "v"(a.l[3]), "v"(b.l[10]), "v"(a.l[4]), "v"(b.l[9]), "v"(a.l[5]), "v"(b.l[8]), "v"(a.l[6]), "v"(b.l[7]), "v"(a.l[7]), "v"(b.l[6]), "v"(a.l[8]), "v"(b.l[5]), "v"(a.l[9]), "v"(b.l[4]), "v"(a.l[10]), "v"(b.l[3]), "v"(a.l[11]), "v"(b.l[2]), "v"(m2), "s"(P11), "v"(m3), "s"(P10), "v"(m4), "s"(P9), "v"(m5), "s"(P8), "v"(m6), "s"(P7), "v"(m7), "s"(P6), "v"(m8), "s"(P5), "v"(m9), "s"(P4), "v"(m10), "s"(P3), "v"(m11), "s"(P2)
        : "vcc");
    { uint64_t s = acc0 + acc1; c20 = c20 + c21 + (uint32_t)(s < acc0); acc0 = s; acc1 = 0; c21 = 0; }
    t[1] = (uint32_t)acc0;
    acc0 = (acc0 >> 32) | ((uint64_t)c20 << 32); c20 = 0;
    asm volatile("v_mad_u64_u32 %0, %4, %6, %7, %0\n\tv_mad_u64_u32 %1, %5, %8, %9, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %10, %11, %0\n\tv_mad_u64_u32 %1, %5, %12, %13, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %14, %15, %0\n\tv_mad_u64_u32 %1, %5, %16, %17, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %18, %19, %0\n\tv_mad_u64_u32 %1, %5, %20, %21, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %22, %23, %0\n\tv_mad_u64_u32 %1, %5, %24, %25, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %26, %27, %0\n\tv_mad_u64_u32 %1, %5, %28, %29, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %30, %31, %0\n\tv_mad_u64_u32 %1, %5, %32, %33, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %34, %35, %0\n\tv_mad_u64_u32 %1, %5, %36, %37, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %38, %39, %0\n\tv_mad_u64_u32 %1, %5, %40, %41, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5"
        : "+&v"(acc0), "+&v"(acc1), "+&v"(c20), "+&v"(c21), "=&s"(sc0), "=&s"(sc1)
        : "v"(a.l[3]), "v"(b.l[11]), "v"(a.l[4]), "v"(b.l[10]), "v"(a.l[5]), "v"(b.l[9]), "v"(a.l[6]), "v"(b.l[8]), "v"(a.l[7]), "v"(b.l[7]), "v"(a.l[8]), "v"(b.l[6]), "v"(a.l[9]), "v"(b.l[5]), "v"(a.l[10]), "v"(b.l[4]), "v"(a.l[11]), "v"(b.l[3]), "v"(m3), "s"(P11), "v"(m4), "s"(P10), "v"(m5), "s"(P9), "v"(m6), "s"(P8), "v"(m7), "s"(P7), "v"(m8), "s"(P6), "v"(m9), "s"(P5), "v"(m10), "s"(P4), "v"(m11), "s"(P3)
        : "vcc");
    { uint64_t s = acc0 + acc1; c20 = c20 + c21 + (uint32_t)(s < acc0); acc0 = s; acc1 = 0; c21 = 0; }
    t[2] = (uint32_t)acc0;
    acc0 = (acc0 >> 32) | ((uint64_t)c20 << 32); c20 = 0;
    asm volatile("v_mad_u64_u32 %0, %4, %6, %7, %0\n\tv_mad_u64_u32 %1, %5, %8, %9, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %10, %11, %0\n\tv_mad_u64_u32 %1, %5, %12, %13, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %14, %15, %0\n\tv_mad_u64_u32 %1, %5, %16, %17, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %18, %19, %0\n\tv_mad_u64_u32 %1, %5, %20, %21, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %22, %23, %0\n\tv_mad_u64_u32 %1, %5, %24, %25, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %26, %27, %0\n\tv_mad_u64_u32 %1, %5, %28, %29, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %30, %31, %0\n\tv_mad_u64_u32 %1, %5, %32, %33, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %34, %35, %0\n\tv_mad_u64_u32 %1, %5, %36, %37, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5"
        : "+&v"(acc0), "+&v"(acc1), "+&v"(c20), "+&v"(c21), "=&s"(sc0), "=&s"(sc1)
        : "v"(a.l[4]), "v"(b.l[11]), "v"(a.l[5]), "v"(b.l[10]), "v"(a.l[6]), "v"(b.l[9]), "v"(a.l[7]), "v"(b.l[8]), "v"(a.l[8]), "v"(b.l[7]), "v"(a.l[9]), "v"(b.l[6]), "v"(a.l[10]), "v"(b.l[5]), "v"(a.l[11]), "v"(b.l[4]), "v"(m4), "s"(P11), "v"(m5), "s"(P10), "v"(m6), "s"(P9), "v"(m7), "s"(P8), "v"(m8), "s"(P7), "v"(m9), "s"(P6), "v"(m10), "s"(P5), "v"(m11), "s"(P4)
        : "vcc");
    { uint64_t s = acc0 + acc1; c20 = c20 + c21 + (uint32_t)(s < acc0); acc0 = s; acc1 = 0; c21 = 0; }
    t[3] = (uint32_t)acc0;
    acc0 = (acc0 >> 32) | ((uint64_t)c20 << 32); c20 = 0;
    asm volatile("v_mad_u64_u32 %0, %4, %6, %7, %0\n\tv_mad_u64_u32 %1, %5, %8, %9, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %10, %11, %0\n\tv_mad_u64_u32 %1, %5, %12, %13, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %14, %15, %0\n\tv_mad_u64_u32 %1, %5, %16, %17, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %18, %19, %0\n\tv_mad_u64_u32 %1, %5, %20, %21, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %22, %23, %0\n\tv_mad_u64_u32 %1, %5, %24, %25, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %26, %27, %0\n\tv_mad_u64_u32 %1, %5, %28, %29, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %30, %31, %0\n\tv_mad_u64_u32 %1, %5, %32, %33, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5"
        : "+&v"(acc0), "+&v"(acc1), "+&v"(c20), "+&v"(c21), "=&s"(sc0), "=&s"(sc1)
        : "v"(a.l[5]), "v"(b.l[11]), "v"(a.l[6]), "v"(b.l[10]), "v"(a.l[7]), "v"(b.l[9]), "v"(a.l[8]), "v"(b.l[8]), "v"(a.l[9]), "v"(b.l[7]), "v"(a.l[10]), "v"(b.l[6]), "v"(a.l[11]), "v"(b.l[5]), "v"(m5), "s"(P11), "v"(m6), "s"(P10), "v"(m7), "s"(P9), "v"(m8), "s"(P8), "v"(m9), "s"(P7), "v"(m10), "s"(P6), "v"(m11), "s"(P5)
        : "vcc");
    { uint64_t s = acc0 + acc1; c20 = c20 + c21 + (uint32_t)(s < acc0); acc0 = s; acc1 = 0; c21 = 0; }
    t[4] = (uint32_t)acc0;
    acc0 = (acc0 >> 32) | ((uint64_t)c20 << 32); c20 = 0;
    asm volatile("v_mad_u64_u32 %0, %4, %6, %7, %0\n\tv_mad_u64_u32 %1, %5, %8, %9, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %10, %11, %0\n\tv_mad_u64_u32 %1, %5, %12, %13, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %14, %15, %0\n\tv_mad_u64_u32 %1, %5, %16, %17, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %18, %19, %0\n\tv_mad_u64_u32 %1, %5, %20, %21, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %22, %23, %0\n\tv_mad_u64_u32 %1, %5, %24, %25, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %26, %27, %0\n\tv_mad_u64_u32 %1, %5, %28, %29, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5"
        : "+&v"(acc0), "+&v"(acc1), "+&v"(c20), "+&v"(c21), "=&s"(sc0), "=&s"(sc1)
        : "v"(a.l[6]), "v"(b.l[11]), "v"(a.l[7]), "v"(b.l[10]), "v"(a.l[8]), "v"(b.l[9]), "v"(a.l[9]), "v"(b.l[8]), "v"(a.l[10]), "v"(b.l[7]), "v"(a.l[11]), "v"(b.l[6]), "v"(m6), "s"(P11), "v"(m7), "s"(P10), "v"(m8), "s"(P9), "v"(m9), "s"(P8), "v"(m10), "s"(P7), "v"(m11), "s"(P6)
        : "vcc");
    { uint64_t s = acc0 + acc1; c20 = c20 + c21 + (uint32_t)(s < acc0); acc0 = s; acc1 = 0; c21 = 0; }
    t[5] = (uint32_t)acc0;
    acc0 = (acc0 >> 32) | ((uint64_t)c20 << 32); c20 = 0;
    asm volatile("v_mad_u64_u32 %0, %4, %6, %7, %0\n\tv_mad_u64_u32 %1, %5, %8, %9, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %10, %11, %0\n\tv_mad_u64_u32 %1, %5, %12, %13, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %14, %15, %0\n\tv_mad_u64_u32 %1, %5, %16, %17, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %18, %19, %0\n\tv_mad_u64_u32 %1, %5, %20, %21, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %22, %23, %0\n\tv_mad_u64_u32 %1, %5, %24, %25, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5"
        : "+&v"(acc0), "+&v"(acc1), "+&v"(c20), "+&v"(c21), "=&s"(sc0), "=&s"(sc1)
        : "v"(a.l[7]), "v"(b.l[11]), "v"(a.l[8]), "v"(b.l[10]), "v"(a.l[9]), "v"(b.l[9]), "v"(a.l[10]), "v"(b.l[8]), "v"(a.l[11]), "v"(b.l[7]), "v"(m7), "s"(P11), "v"(m8), "s"(P10), "v"(m9), "s"(P9), "v"(m10), "s"(P8), "v"(m11), "s"(P7)
        : "vcc");
    { uint64_t s = acc0 + acc1; c20 = c20 + c21 + (uint32_t)(s < acc0); acc0 = s; acc1 = 0; c21 = 0; }
    t[6] = (uint32_t)acc0;
    acc0 = (acc0 >> 32) | ((uint64_t)c20 << 32); c20 = 0;
    asm volatile("v_mad_u64_u32 %0, %4, %6, %7, %0\n\tv_mad_u64_u32 %1, %5, %8, %9, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %10, %11, %0\n\tv_mad_u64_u32 %1, %5, %12, %13, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %14, %15, %0\n\tv_mad_u64_u32 %1, %5, %16, %17, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %18, %19, %0\n\tv_mad_u64_u32 %1, %5, %20, %21, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5"
        : "+&v"(acc0), "+&v"(acc1), "+&v"(c20), "+&v"(c21), "=&s"(sc0), "=&s"(sc1)
        : "v"(a.l[8]), "v"(b.l[11]), "v"(a.l[9]), "v"(b.l[10]), "v"(a.l[10]), "v"(b.l[9]), "v"(a.l[11]), "v"(b.l[8]), "v"(m8), "s"(P11), "v"(m9), "s"(P10), "v"(m10), "s"(P9), "v"(m11), "s"(P8)
        : "vcc");
    { uint64_t s = acc0 + acc1; c20 = c20 + c21 + (uint32_t)(s < acc0); acc0 = s; acc1 = 0; c21 = 0; }
    t[7] = (uint32_t)acc0;
    acc0 = (acc0 >> 32) | ((uint64_t)c20 << 32); c20 = 0;
    asm volatile("v_mad_u64_u32 %0, %4, %6, %7, %0\n\tv_mad_u64_u32 %1, %5, %8, %9, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %10, %11, %0\n\tv_mad_u64_u32 %1, %5, %12, %13, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %14, %15, %0\n\tv_mad_u64_u32 %1, %5, %16, %17, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5"
        : "+&v"(acc0), "+&v"(acc1), "+&v"(c20), "+&v"(c21), "=&s"(sc0), "=&s"(sc1)
        : "v"(a.l[9]), "v"(b.l[11]), "v"(a.l[10]), "v"(b.l[10]), "v"(a.l[11]), "v"(b.l[9]), "v"(m9), "s"(P11), "v"(m10), "s"(P10), "v"(m11), "s"(P9)
        : "vcc");
    { uint64_t s = acc0 + acc1; c20 = c20 + c21 + (uint32_t)(s < acc0); acc0 = s; acc1 = 0; c21 = 0; }
    t[8] = (uint32_t)acc0;
    acc0 = (acc0 >> 32) | ((uint64_t)c20 << 32); c20 = 0;
    asm volatile("v_mad_u64_u32 %0, %4, %6, %7, %0\n\tv_mad_u64_u32 %1, %5, %8, %9, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5\n\tv_mad_u64_u32 %0, %4, %10, %11, %0\n\tv_mad_u64_u32 %1, %5, %12, %13, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5"
        : "+&v"(acc0), "+&v"(acc1), "+&v"(c20), "+&v"(c21), "=&s"(sc0), "=&s"(sc1)
        : "v"(a.l[10]), "v"(b.l[11]), "v"(a.l[11]), "v"(b.l[10]), "v"(m10), "s"(P11), "v"(m11), "s"(P10)
        : "vcc");
    { uint64_t s = acc0 + acc1; c20 = c20 + c21 + (uint32_t)(s < acc0); acc0 = s; acc1 = 0; c21 = 0; }
    t[9] = (uint32_t)acc0;
    acc0 = (acc0 >> 32) | ((uint64_t)c20 << 32); c20 = 0;
    asm volatile("v_mad_u64_u32 %0, %4, %6, %7, %0\n\tv_mad_u64_u32 %1, %5, %8, %9, %1\n\tv_addc_co_u32_e64 %2, vcc, 0, %2, %4\n\tv_addc_co_u32_e64 %3, vcc, 0, %3, %5"
        : "+&v"(acc0), "+&v"(acc1), "+&v"(c20), "+&v"(c21), "=&s"(sc0), "=&s"(sc1)
        : "v"(a.l[11]), "v"(b.l[11]), "v"(m11), "s"(P11)
        : "vcc");
    { uint64_t s = acc0 + acc1; c20 = c20 + c21 + (uint32_t)(s < acc0); acc0 = s; acc1 = 0; c21 = 0; }
    t[10] = (uint32_t)acc0;
    acc0 = (acc0 >> 32) | ((uint64_t)c20 << 32); c20 = 0;
  t[11] = (uint32_t)acc0;
  red(r, t);
}

template <int V, int LDSB>
__global__ void __launch_bounds__(64) k_fpmul(uint32_t *out, uint32_t iters, uint32_t seed) {
  __shared__ uint32_t pad[LDSB ? LDSB : 1];
  fpv x, y;
#pragma unroll
  for (int i = 0; i < 12; i++) { y.l[i] = (seed * 2654435761u + i * 97 + threadIdx.x) & 0x0fffffff; x.l[i] = (seed + i * 31 + blockIdx.x) & 0x0fffffff; }
  for (uint32_t it = 0; it < iters; it++) { if (V == 0) mul_single(x, x, y); else mul_dual(x, x, y); }
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) acc ^= x.l[i];
  if (LDSB) { pad[threadIdx.x] = acc; __syncthreads(); acc ^= pad[(threadIdx.x + 1) & 63]; }
  out[blockIdx.x * 64 + threadIdx.x] = acc;
}
template <int V, int LDSB> void run(const char *name, unsigned blocks, uint32_t *sink) {
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  k_fpmul<V, LDSB><<<blocks, 64>>>(sink, 16, 1);
  hipEventRecord(a);
  k_fpmul<V, LDSB><<<blocks, 64>>>(sink, 512, 3);
  hipEventRecord(b); hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  double per_wave_us = ms * 1e3 / 512.0;
  printf("%-7s blocks=%6u lds=%6d: %.3f ms, %.3e Fp-mul/s, per-wave mul latency %.3f us\n", name, blocks, LDSB, ms,
         (double)blocks * 64 * 512 / (ms * 1e-3), per_wave_us);
}
int main() {
  uint32_t *sink; hipMalloc(&sink, 1 << 24);
  // 1 wave per SIMD: 1024 single-wave blocks, 36 KB LDS each (4 per CU)
  run<0, 9216>("single", 1024, sink);
  run<1, 9216>("dual", 1024, sink);
  run<0, 9216>("single", 64, sink);
  run<1, 9216>("dual", 64, sink);
  // high occupancy
  run<0, 0>("single", 16384, sink);
  run<1, 0>("dual", 16384, sink);
  printf("status %s\n", hipGetErrorString(hipDeviceSynchronize()));
}