// Wave-per-point G2 engine (grandine_amd/csrc/bls_w4.h) on MI355X: every formula against the
// engine's one-lane formulas (bls_curve.h / bls_hash.h / bls_pairing.h) on points r G2, plus
// the latency of the chains the latency regime runs (doubling, cofactor clearing, Miller
// lines).
// With a file argument it also writes every W4 result (engine words) for the independent
// Python-integer check tools/ubench/w4_check.py (oracle/bls12_381.py arithmetic).
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -o tools/ubench/_bin/w4_check tools/ubench/w4_check.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "../../grandine_amd/csrc/gbls_common.h"
#include "../../grandine_amd/csrc/bls_w4.h"

using namespace gbls;

#define CHK(x)                                                                  \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

__device__ g2a gen2() {
  g2a g;
  g.x = fp2_const(k::G2X_C0, k::G2X_C1);
  g.y = fp2_const(k::G2Y_C0, k::G2Y_C1);
  return g;
}
// engine-form Jacobian copy of a row-form point (two rounds of canonical stores)
__device__ void store_j(const w4::Ctx &c, g2j *o, const w4::J &p) {
  __shared__ uint32_t dummy[2][12];
  w4::store4(c, p.x.c0, p.x.c1, p.y.c0, p.y.c1, o->x.c0.l, o->x.c1.l, o->y.c0.l, o->y.c1.l);
  w4::store4(c, p.z.c0, p.z.c1, p.z.c0, p.z.c1, o->z.c0.l, o->z.c1.l, dummy[0], dummy[1]);
  __syncthreads();
}

// failure bits per wave: 1 gather, 2 dbl, 4 add, 8 add(P,P), 16 add(P,-P), 32 add(inf,Q),
// 64 psi, 128 psi2, 256 [|x|]P, 512 clear, 1024 affine of clear, 2048 line_dbl, 4096 line_add,
// 8192 madd, 16384 32-bit scalar chain, 32768 projective addition step
// Dump slots (w4_check DUMPFILE: every W4 result, engine words, for tools/ubench/w4_check.py's
// independent Python-integer recomputation from the seeds): see DUMP_NAMES there.
constexpr int kDumpSlots = 16;
__device__ void dump_words(uint32_t *dst, const void *src, int nwords) {
  const uint32_t *w = reinterpret_cast<const uint32_t *>(src);
  for (int i = threadIdx.x; i < nwords; i += 64) dst[i] = w[i];
}
__global__ void __launch_bounds__(64) k_check(const uint64_t *seeds, uint32_t *fails, g2j *dump) {
  w4::Ctx c;
  w4::init(c);
  __shared__ g2j out;
  __shared__ g2a outa;
  uint32_t f = 0;
  g2j *dd = dump ? dump + (size_t)blockIdx.x * kDumpSlots : nullptr;
  auto put = [&](int slot, const void *v, int nwords) {
    __syncthreads();
    if (dd) dump_words(reinterpret_cast<uint32_t *>(dd + slot), v, nwords);
    __syncthreads();
  };
  // gather
  {
    uint32_t o0, o1, o2, o3;
    w4::gather(threadIdx.x, o0, o1, o2, o3);
    const uint32_t j = threadIdx.x & 15;
    if (o0 != j || o1 != 16 + j || o2 != 32 + j || o3 != 48 + j) f |= 1;
  }
  const uint64_t s = seeds[blockIdx.x];
  g2j P, Q, R;
  mul_u64(P, gen2(), s | 1);
  mul_u64(Q, gen2(), (s >> 7) * 3 + 5);
  w4::J jp, jq, jr;
  w4::load(c, jp, P);
  w4::load(c, jq, Q);
  auto same = [&](const g2j &want) {
    return jac_eq(out, want);
  };
  // dbl
  w4::dbl(c, jr, jp);
  store_j(c, &out, jr);
  put(0, &out, 72);
  jac_dbl(R, P);
  if (!same(R)) f |= 2;
  // add
  w4::add(c, jr, jp, jq);
  store_j(c, &out, jr);
  put(1, &out, 72);
  jac_add(R, P, Q);
  if (!same(R)) f |= 4;
  w4::add(c, jr, jp, jp);
  store_j(c, &out, jr);
  put(2, &out, 72);
  jac_dbl(R, P);
  if (!same(R)) f |= 8;
  {
    w4::J jn;
    w4::negy<10, 10>(c, jn, jp);
    w4::add(c, jr, jp, jn);
    store_j(c, &out, jr);
    if (!jac_is_inf(out)) f |= 16;
    w4::J ji;
    w4::set_inf(c, ji);
    w4::add(c, jr, ji, jq);
    store_j(c, &out, jr);
    if (!same(Q)) f |= 32;
  }
  w4::psi<10>(c, jr, jp);
  store_j(c, &out, jr);
  put(3, &out, 72);
  g2_psi(R, P);
  if (!same(R)) f |= 64;
  w4::psi2(c, jr, jp);
  store_j(c, &out, jr);
  put(4, &out, 72);
  g2_psi2(R, P);
  if (!same(R)) f |= 128;
  w4::mul_by_xabs(c, jr, jp);
  store_j(c, &out, jr);
  put(5, &out, 72);
  mul_by_xabs(R, P);
  if (!same(R)) f |= 256;
  w4::clear_cofactor(c, jr, jp);
  store_j(c, &out, jr);
  put(6, &out, 72);
  clear_cofactor_g2(R, P);
  if (!same(R)) f |= 512;
  w4::store_affine(c, &outa, jr);
  __syncthreads();
  put(7, &outa, 48);
  {
    g2a want;
    jac_to_aff(want, R);
    bool eq = fp2_eq(want.x, outa.x) && fp2_eq(want.y, outa.y);
    if (!eq) f |= 1024;
  }
  // Miller steps from the affine point Q: T = (x, y, 1) homogeneous, then doubling and addition
  {
    g2a qa;
    jac_to_aff(qa, Q);
    g2h T;
    T.x = qa.x;
    T.y = qa.y;
    fp2_one(T.z);
    jac_dbl(R, P);  // a second affine point for the addition step
    g2a ra;
    jac_to_aff(ra, R);
    w4::J jt;
    w4::A2 jra;
    {
      g2j tj;
      tj.x = T.x;
      tj.y = T.y;
      tj.z = T.z;
      w4::load(c, jt, tj);
      w4::load(c, jra, ra);
    }
    fp2 L0, L2, L3;
    w4::f2 l0, l2, l3;
    line_dbl(T, L0, L2, L3);
    w4::line_dbl(c, jt, l0, l2, l3);
    __shared__ fp2 ll[3];
    __shared__ g2j tt;
    w4::store4(c, l0.c0, l0.c1, l2.c0, l2.c1, ll[0].c0.l, ll[0].c1.l, ll[1].c0.l, ll[1].c1.l);
    w4::store4(c, l3.c0, l3.c1, l3.c0, l3.c1, ll[2].c0.l, ll[2].c1.l, ll[2].c0.l, ll[2].c1.l);
    store_j(c, &tt, jt);
    __syncthreads();
    put(8, &tt, 72);
    put(9, ll, 72);
    // the row engine keeps the lane formulas' exact values mod p
    if (!(fp2_eq(ll[0], L0) && fp2_eq(ll[1], L2) && fp2_eq(ll[2], L3) && fp2_eq(tt.x, T.x) &&
          fp2_eq(tt.y, T.y) && fp2_eq(tt.z, T.z)))
      f |= 2048;
    line_add_aff(T, ra, L0, L2, L3);
    w4::line_add_aff(c, jt, jra, l0, l2, l3);
    __syncthreads();
    w4::store4(c, l0.c0, l0.c1, l2.c0, l2.c1, ll[0].c0.l, ll[0].c1.l, ll[1].c0.l, ll[1].c1.l);
    w4::store4(c, l3.c0, l3.c1, l3.c0, l3.c1, ll[2].c0.l, ll[2].c1.l, ll[2].c0.l, ll[2].c1.l);
    store_j(c, &tt, jt);
    __syncthreads();
    put(10, &tt, 72);
    put(11, ll, 72);
    if (!(fp2_eq(ll[0], L0) && fp2_eq(ll[1], L2) && fp2_eq(ll[2], L3) && fp2_eq(tt.x, T.x) &&
          fp2_eq(tt.y, T.y) && fp2_eq(tt.z, T.z)))
      f |= 4096;
  }
  // madd against jac_add_aff, and a 32-bit scalar chain against mul_u64
  {
    g2a qa;
    jac_to_aff(qa, Q);
    w4::A2 jqa;
    w4::load(c, jqa, qa);
    w4::madd(c, jr, jp, jqa);
    store_j(c, &out, jr);
    put(12, &out, 72);
    jac_add_aff(R, P, qa);
    if (!same(R)) f |= 8192;
    const uint64_t k = (s * 0x2545F4914F6CDD1Dull) >> 32 | 1;
    w4::J acc;
    acc.x = jqa.x;
    acc.y = jqa.y;
    acc.z = {c.one, 0u};
    const int top = 63 - __clzll((long long)k);
    for (int bit = top - 1; bit >= 0; bit--) {
      w4::dbl(c, acc, acc);
      if ((k >> bit) & 1) w4::madd(c, acc, acc, jqa);
    }
    store_j(c, &out, acc);
    put(13, &out, 72);
    mul_u64(R, qa, k);
    if (!same(R)) f |= 16384;
  }
  // projective addition step: Q Jacobian -> homogeneous, T from a doubling of Q; the same point
  // and proportional lines as the affine step (the lines carry an Fp2 factor)
  {
    g2a qa;
    jac_to_aff(qa, Q);
    g2h T;
    T.x = qa.x;
    T.y = qa.y;
    fp2_one(T.z);
    fp2 L0, L2, L3;
    line_dbl(T, L0, L2, L3);
    w4::J qh, jt;
    w4::jac_to_hom(c, qh, jq);
    {
      g2j tj;
      tj.x = T.x;
      tj.y = T.y;
      tj.z = T.z;
      w4::load(c, jt, tj);
    }
    line_add_aff(T, qa, L0, L2, L3);
    w4::f2 l0, l2, l3;
    w4::line_add_proj(c, jt, qh, l0, l2, l3);
    __shared__ fp2 ll[3];
    __shared__ g2j tt;
    w4::store4(c, l0.c0, l0.c1, l2.c0, l2.c1, ll[0].c0.l, ll[0].c1.l, ll[1].c0.l, ll[1].c1.l);
    w4::store4(c, l3.c0, l3.c1, l3.c0, l3.c1, ll[2].c0.l, ll[2].c1.l, ll[2].c0.l, ll[2].c1.l);
    store_j(c, &tt, jt);
    __syncthreads();
    put(14, &tt, 72);
    put(15, ll, 72);
    fp2 a, b;
    bool ok = true;
    // same homogeneous point: X Z' = X' Z, Y Z' = Y' Z
    fp2_mul(a, tt.x, T.z); fp2_mul(b, T.x, tt.z); ok &= fp2_eq(a, b);
    fp2_mul(a, tt.y, T.z); fp2_mul(b, T.y, tt.z); ok &= fp2_eq(a, b);
    // proportional lines: l0 L2 = L0 l2, l3 L2 = L3 l2
    fp2_mul(a, ll[0], L2); fp2_mul(b, L0, ll[1]); ok &= fp2_eq(a, b);
    fp2_mul(a, ll[2], L2); fp2_mul(b, L3, ll[1]); ok &= fp2_eq(a, b);
    if (!ok) f |= 32768;
  }
  if (threadIdx.x == 0) fails[blockIdx.x] = f;
}

// latency of the cofactor clearing + affine conversion per wave, and of 1000 doublings
__global__ void __launch_bounds__(64) k_time(const uint64_t *seeds, g2a *out, uint64_t *cyc) {
  w4::Ctx c;
  w4::init(c);
  g2j P;
  mul_u64(P, gen2(), seeds[blockIdx.x] | 1);
  w4::J jp, jr;
  w4::load(c, jp, P);
  uint64_t t0 = wall_clock64();
  for (int i = 0; i < 1000; i++) w4::dbl(c, jp, jp);
  uint64_t t1 = wall_clock64();
  w4::clear_cofactor(c, jr, jp);
  uint64_t t2 = wall_clock64();
  w4::store_affine(c, out + blockIdx.x, jr);
  uint64_t t3 = wall_clock64();
  w4::J jt = jr;
  w4::f2 l0, l2, l3;
  uint32_t acc = 0;
  for (int e = 0; e < 63; e++) {
    w4::line_dbl(c, jt, l0, l2, l3);
    acc += l0.c0 ^ l2.c1 ^ l3.c0;
  }
  uint64_t t4 = wall_clock64();
  if (threadIdx.x == 0) {
    cyc[4 * blockIdx.x] = t1 - t0;
    cyc[4 * blockIdx.x + 1] = t2 - t1;
    cyc[4 * blockIdx.x + 2] = t3 - t2;
    cyc[4 * blockIdx.x + 3] = (t4 - t3) + (acc == 0x12345 ? 1 : 0);
  }
}

int main(int argc, char **argv) {
  const int n = 64;
  uint64_t hs[n];
  for (int i = 0; i < n; i++) hs[i] = 0x9E3779B97F4A7C15ull * (i + 1) ^ (0xabcdefull << (i % 17));
  uint64_t *ds;
  uint32_t *df;
  CHK(hipMalloc(&ds, sizeof hs));
  CHK(hipMalloc(&df, n * 4));
  CHK(hipMemcpy(ds, hs, sizeof hs, hipMemcpyHostToDevice));
  g2j *ddump = nullptr;
  if (argc > 1) CHK(hipMalloc(&ddump, (size_t)n * kDumpSlots * sizeof(g2j)));
  k_check<<<n, 64>>>(ds, df, ddump);
  CHK(hipDeviceSynchronize());
  if (ddump) {  // the seeds, then every block's slots (tools/ubench/w4_check.py)
    const size_t bytes = (size_t)n * kDumpSlots * sizeof(g2j);
    void *h = malloc(bytes);
    CHK(hipMemcpy(h, ddump, bytes, hipMemcpyDeviceToHost));
    FILE *fo = fopen(argv[1], "wb");
    if (!fo || fwrite(hs, sizeof hs, 1, fo) != 1 || fwrite(h, bytes, 1, fo) != 1) {
      fprintf(stderr, "cannot write %s\n", argv[1]);
      return 2;
    }
    fclose(fo);
    free(h);
  }
  uint32_t hf[n];
  CHK(hipMemcpy(hf, df, sizeof hf, hipMemcpyDeviceToHost));
  int bad = 0;
  uint32_t orf = 0;
  for (int i = 0; i < n; i++) {
    if (hf[i]) bad++;
    orf |= hf[i];
  }
  printf("check: %d / %d points with a mismatch (failure bits OR = 0x%x)\n", bad, n, orf);
  g2a *dout;
  uint64_t *dc;
  CHK(hipMalloc(&dout, n * sizeof(g2a)));
  CHK(hipMalloc(&dc, n * 4 * 8));
  for (int rep = 0; rep < 2; rep++) {
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    CHK(hipEventRecord(e0));
    k_time<<<n, 64>>>(ds, dout, dc);
    CHK(hipEventRecord(e1));
    CHK(hipDeviceSynchronize());
    float ms;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    uint64_t hc[n * 4];
    CHK(hipMemcpy(hc, dc, sizeof hc, hipMemcpyDeviceToHost));
    double s[4] = {0, 0, 0, 0};
    for (int i = 0; i < n; i++)
      for (int k = 0; k < 4; k++) s[k] += hc[4 * i + k];
    // wall_clock64 runs at 100 MHz
    printf("w4 (64 waves): dbl %.3f us each; clear_cofactor %.1f us; to affine %.1f us; 63 line_dbl %.1f us (%.2f us each); kernel %.3f ms\n",
           s[0] / n / 1000 * 0.01, s[1] / n * 0.01, s[2] / n * 0.01, s[3] / n * 0.01, s[3] / n * 0.01 / 63, ms);
  }
  return bad ? 1 : 0;
}
