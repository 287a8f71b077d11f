// bls_w4.h primitives one by one on MI355X (debug aid): every value of a fixed list of
// operations on random operands, written canonical (engine words); tools/ubench/w4_prim.py
// recomputes them with Python integers.
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -o tools/ubench/_bin/w4_prim tools/ubench/w4_prim.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "../../grandine_amd/csrc/bls_w4.h"

using namespace gbls;
constexpr int NOUT = 84;
namespace gbls { namespace w4 {
__device__ __noinline__ void dbl_t(const Ctx &c, J &o, const J &p, uint32_t *dv) {
  uint32_t a0, ax, b0, bx;
  mul4(c, a0, ax, b0, bx, add(p.x.c0, p.x.c1), sub<10>(c, p.x.c0, p.x.c1), p.x.c0, p.x.c1,
       add(p.y.c0, p.y.c1), sub<10>(c, p.y.c0, p.y.c1), p.y.c0, p.y.c1);
  const f2 A = sqr_of(a0, ax), B = sqr_of(b0, bx);
  const f2 E = small(A, 3);
  uint32_t c0, cx, f0, fx;
  mul4(c, c0, cx, f0, fx, add(B.c0, B.c1), sub<2>(c, B.c0, B.c1), B.c0, B.c1, add(E.c0, E.c1),
       sub<3>(c, E.c0, E.c1), E.c0, E.c1);
  const f2 C = sqr_of(c0, cx), F = sqr_of(f0, fx);
  const f2 t = add(p.x, B);
  uint32_t g0, gx, yz0, yz1;
  mul4(c, g0, gx, yz0, yz1, add(t.c0, t.c1), sub<10>(c, t.c0, t.c1), t.c0, t.c1, p.y.c0, p.z.c0,
       p.y.c1, p.z.c1);
  const f2 XB2 = sqr_of(g0, gx);
  const f2 D = small(sub<2, 3>(c, XB2, add(A, C)), 2);
  const f2 X3 = sub<5, 6>(c, F, small(D, 2));
  const f2 u = sub<6, 7>(c, D, X3);
  uint32_t m0, m1, m2, yz2;
  mul4(c, m0, m1, m2, yz2, E.c0, u.c0, E.c1, u.c1, add(E.c0, E.c1), add(u.c0, u.c1),
       add(p.y.c0, p.y.c1), add(p.z.c0, p.z.c1));
  const f2 Eu = kara(c, m0, m1, m2);
  const f2 YZ = kara(c, yz0, yz1, yz2);
  dv[0] = A.c1; dv[1] = C.c1; dv[2] = F.c1; dv[3] = XB2.c1; dv[4] = D.c1; dv[5] = X3.c1;
  o.x = X3;
  o.y = sub<4, 5>(c, Eu, small(C, 8));
  o.z = small(YZ, 2);
}
} }  // namespace gbls::w4
constexpr int NIN = 12;

// in: 4 Fp per wave (a0, a1, b0, b1) as engine words; out: NOUT values per wave
__global__ void __launch_bounds__(64) k_prim(const fp *in, fp *out) {
  w4::Ctx c;
  w4::init(c);
  const fp *x = in + NIN * blockIdx.x;
  const uint32_t cin = dfp::konst(dfp::K_CIN);
  uint32_t a0, a1, b0, b1;
  w4::mul4(c, a0, a1, b0, b1, w4::repack(x[0], c.t.j), cin, w4::repack(x[1], c.t.j), cin,
           w4::repack(x[2], c.t.j), cin, w4::repack(x[3], c.t.j), cin);
  uint32_t v[NOUT];
  uint32_t d;
  // 0: a0 b0 (row 0), 1: a1 b1 (row 3)
  w4::mul4(c, v[0], d, d, v[1], a0, b0, a1, a1, a1, a1, a1, b1);
  // 2-3: Karatsuba (a0 + a1 u)(b0 + b1 u)
  uint32_t t0, t1, t2;
  w4::mul4(c, t0, t1, t2, d, a0, b0, a1, b1, w4::add(a0, a1), w4::add(b0, b1), a0, b0);
  const w4::f2 k = w4::kara(c, t0, t1, t2);
  v[2] = k.c0;
  v[3] = k.c1;
  // 4-5: squaring of a
  uint32_t s0, s1;
  w4::mul4(c, s0, s1, d, d, w4::add(a0, a1), w4::sub<2>(c, a0, a1), a0, a1, a0, a1, a0, a1);
  const w4::f2 sq = w4::sqr_of(s0, s1);
  v[4] = sq.c0;
  v[5] = sq.c1;
  // 6-15: sub<K>(a0, b0) for K = 1..10
  v[6] = w4::sub<1>(c, a0, b0);
  v[7] = w4::sub<2>(c, a0, b0);
  v[8] = w4::sub<3>(c, a0, b0);
  v[9] = w4::sub<4>(c, a0, b0);
  v[10] = w4::sub<5>(c, a0, b0);
  v[11] = w4::sub<6>(c, a0, b0);
  v[12] = w4::sub<7>(c, a0, b0);
  v[13] = w4::sub<8>(c, a0, b0);
  v[14] = w4::sub<9>(c, a0, b0);
  v[15] = w4::sub<10>(c, a0, b0);
  v[16] = w4::small(a0, 3);
  v[17] = w4::small(a1, 8);
  v[18] = w4::half(c, a0);
  v[19] = w4::add(a0, b1);
  // 20: (3 a0) * (sub<3>(a1, b1)) ; 21: product of sums of 8 a0
  uint32_t p0, p1;
  w4::mul4(c, p0, p1, d, d, w4::small(a0, 3), w4::sub<3>(c, a1, b1), w4::small(a0, 8), w4::small(b0, 8),
           a0, a0, a0, a0);
  v[20] = p0;
  v[21] = p1;
  v[22] = c.bias[0];
  v[23] = c.bias[9];
  // 24-29: dbl(P), 30-35: add(P, Q); P = (x0..x5), Q = (x6..x11) as Jacobian Fp2 coordinates
  {
    g2j P, Q;
    P.x.c0 = x[0]; P.x.c1 = x[1]; P.y.c0 = x[2]; P.y.c1 = x[3]; P.z.c0 = x[4]; P.z.c1 = x[5];
    Q.x.c0 = x[6]; Q.x.c1 = x[7]; Q.y.c0 = x[8]; Q.y.c1 = x[9]; Q.z.c0 = x[10]; Q.z.c1 = x[11];
    w4::J jp, jq, jr;
    w4::load(c, jp, P);
    w4::load(c, jq, Q);
    w4::dbl(c, jr, jp);
    v[24] = jr.x.c0; v[25] = jr.x.c1; v[26] = jr.y.c0; v[27] = jr.y.c1; v[28] = jr.z.c0; v[29] = jr.z.c1;
    w4::add(c, jr, jp, jq);
    v[30] = jr.x.c0; v[31] = jr.x.c1; v[32] = jr.y.c0; v[33] = jr.y.c1; v[34] = jr.z.c0; v[35] = jr.z.c1;
    // 36..: dbl's intermediates A, B, E, C, F, XB2, D, X3, u, Eu, YZ, 8C (2 each)
    const w4::J &p = jp;
    using namespace w4;
    uint32_t a0, ax, b0, bx;
    mul4(c, a0, ax, b0, bx, add(p.x.c0, p.x.c1), sub<10>(c, p.x.c0, p.x.c1), p.x.c0, p.x.c1,
         add(p.y.c0, p.y.c1), sub<10>(c, p.y.c0, p.y.c1), p.y.c0, p.y.c1);
    const f2 A = sqr_of(a0, ax), B = sqr_of(b0, bx);
    const f2 E = small(A, 3);
    uint32_t c0, cx, f0, fx;
    mul4(c, c0, cx, f0, fx, add(B.c0, B.c1), sub<2>(c, B.c0, B.c1), B.c0, B.c1, add(E.c0, E.c1),
         sub<3>(c, E.c0, E.c1), E.c0, E.c1);
    const f2 C = sqr_of(c0, cx), F = sqr_of(f0, fx);
    const f2 t = add(p.x, B);
    uint32_t g0, gx, yz0, yz1;
    mul4(c, g0, gx, yz0, yz1, add(t.c0, t.c1), sub<10>(c, t.c0, t.c1), t.c0, t.c1, p.y.c0, p.z.c0,
         p.y.c1, p.z.c1);
    const f2 XB2 = sqr_of(g0, gx);
    const f2 D = small(sub<2, 3>(c, XB2, add(A, C)), 2);
    const f2 X3 = sub<5, 6>(c, F, small(D, 2));
    const f2 u = sub<6, 7>(c, D, X3);
    uint32_t m0, m1, m2, yz2;
    mul4(c, m0, m1, m2, yz2, E.c0, u.c0, E.c1, u.c1, add(E.c0, E.c1), add(u.c0, u.c1),
         add(p.y.c0, p.y.c1), add(p.z.c0, p.z.c1));
    const f2 Eu = kara(c, m0, m1, m2);
    const f2 YZ = kara(c, yz0, yz1, yz2);
    const f2 C8 = small(C, 8);
    const f2 all[12] = {A, B, E, C, F, XB2, D, X3, u, Eu, YZ, C8};
    for (int i = 0; i < 12; i++) {
      v[36 + 2 * i] = all[i].c0;
      v[37 + 2 * i] = all[i].c1;
    }
    // 60-65: the copy's outputs; 66-71: a second call of dbl
    const f2 Y3 = sub<4, 5>(c, Eu, small(C, 8)), Z3 = small(YZ, 2);
    v[60] = X3.c0; v[61] = X3.c1; v[62] = Y3.c0; v[63] = Y3.c1; v[64] = Z3.c0; v[65] = Z3.c1;
    w4::J j2;
    w4::dbl(c, j2, jp);
    v[66] = j2.x.c0; v[67] = j2.x.c1; v[68] = j2.y.c0; v[69] = j2.y.c1; v[70] = j2.z.c0; v[71] = j2.z.c1;
    // 72-77: test-file function copy's outputs, 78-83: its intermediates A1 C1 F1 XB2_1 D1 X3_1
    w4::dbl_t(c, j2, jp, v + 78);
    v[72] = j2.x.c0; v[73] = j2.x.c1; v[74] = j2.y.c0; v[75] = j2.y.c1; v[76] = j2.z.c0; v[77] = j2.z.c1;
  }
  __shared__ uint32_t w[NOUT][12];
  for (int i = 0; i < NOUT; i += 4) {
    uint32_t *wp[4] = {w[i], w[i + 1], w[i + 2], w[i + 3]};
    w4::store4(c, v[i], v[i + 1], v[i + 2], v[i + 3], wp[0], wp[1], wp[2], wp[3]);
  }
  __syncthreads();
  if (threadIdx.x < 12)
    for (int i = 0; i < NOUT; i++) out[NOUT * blockIdx.x + i].l[threadIdx.x] = w[i][threadIdx.x];
}

int main(int argc, char **argv) {
  const int n = 16;
  fp *h = (fp *)malloc(NIN * n * sizeof(fp));
  srand(7);
  // random values below 2^380 (< p), engine form = any word string below p
  for (int i = 0; i < NIN * n; i++)
    for (int k = 0; k < 12; k++) h[i].l[k] = (k == 11) ? (rand() & 0x0fffffff) : ((uint32_t)rand() * 2654435761u);
  fp *din, *dout;
  hipMalloc(&din, NIN * n * sizeof(fp));
  hipMalloc(&dout, NOUT * n * sizeof(fp));
  hipMemcpy(din, h, NIN * n * sizeof(fp), hipMemcpyHostToDevice);
  k_prim<<<n, 64>>>(din, dout);
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  fp *o = (fp *)malloc(NOUT * n * sizeof(fp));
  hipMemcpy(o, dout, NOUT * n * sizeof(fp), hipMemcpyDeviceToHost);
  FILE *f = fopen(argc > 1 ? argv[1] : "w4_prim.bin", "wb");
  fwrite(h, sizeof(fp), NIN * n, f);
  fwrite(o, sizeof(fp), NOUT * n, f);
  fclose(f);
  printf("wrote %d waves\n", n);
  return 0;
}
