// Wave-per-point G2 engine for the latency regime (VERDICT r02 "next 1b"): one 64-lane wave
// owns one G2 point; its four 16-lane DPP rows each hold every Fp value of the point in the
// row-distributed form of bls_dfp.h (lane j = limb j, R = 2^448), replicated in all four
// rows.  A "round" is one row-distributed Montgomery product per row -- four independent Fp
// products side by side, operands picked per row with v_cndmask on the row index, results
// shared with the gfx950 v_permlane16_swap / v_permlane32_swap row exchanges -- so the
// dependency DAG of a point formula runs at one row product (~0.46 us on MI355X) per level
// of 4 products instead of one one-lane product (~1.2 us) per Fp product.  Everything else
// (sums, differences, halving, selects) is lane-local and redundant across rows.
//
// Counted in rounds (each ~1 row product):
//   Jacobian doubling dbl-2009-l           4   (16 products; gang_dbl's levels, bls_gang.h)
//   Jacobian addition add-2007-bl         11 + 2 zero tests
//   Miller doubling step (line_dbl)        6   (21 products)
//   Miller addition step (line_add_aff)   10   (37 products)
// against 16 / 43 / 21 / 37 one-lane products.
//
// Value contract (bls_dfp.h): products < 1.0001 p; sub<K>(a, b) = a + 2^K p - b (lower limbs
// pre-borrowed, bls_dfp_tables.h K_BIASK) needs b < 2^K p with margin and gives < a + 2^K p;
// a product input must stay below 2^392 (~2517 p).  Each formula states its output bounds in
// units of p; point coordinates entering a formula must be < 600 p.
//
// Every branch in this file depends only on values all 64 lanes share (one point per wave),
// so it is wave-uniform.
#pragma once
#include "bls_curve.h"
#include "bls_dfp.h"
#include "bls_pairing.h"

namespace gbls {
namespace w4 {

struct Ctx {
  dfp::Tabs t;
  uint32_t r;         // row of this lane in its wave
  uint32_t bias[10];  // this lane's limb of 2^(k+1) p (pre-borrowed)
  uint32_t one;       // limb of 1 (x 2^448)
};
__device__ __forceinline__ void init(Ctx &c) {
  dfp::load_tabs(c.t);
  c.r = (threadIdx.x >> 4) & 3;
#pragma unroll
  for (int k = 0; k < 10; k++) c.bias[k] = dfp::K_BIASK[k][c.t.j];
  c.one = dfp::konst(dfp::K_ONE);
}

// A latency-chain kernel claims its SIMD: the clobbers make it allocate 256 VGPRs + 256 AGPRs
// (occupancy 1), so no wave of a concurrent kernel (the signature / key side streams) is ever
// co-resident and competes for its issue slots.  Used for launches of a few hundred waves.
__device__ __forceinline__ void exclusive_simd() { asm volatile("" ::: "v255", "a255"); }
constexpr uint32_t kExclusiveMaxWaves = 512;

// ---- rows
__device__ __forceinline__ uint32_t sel(const Ctx &c, uint32_t x0, uint32_t x1, uint32_t x2,
                                        uint32_t x3) {
  const uint32_t lo = (c.r & 1) ? x1 : x0;
  const uint32_t hi = (c.r & 1) ? x3 : x2;
  return (c.r & 2) ? hi : lo;
}
// o_k = the value row k holds, in every row
__device__ __forceinline__ void gather(uint32_t p, uint32_t &o0, uint32_t &o1, uint32_t &o2,
                                       uint32_t &o3) {
#if !defined(GBLS_W4_BPERMUTE)
  // permlane16_swap(x, x): {rows (0,0,2,2), rows (1,1,3,3)}; permlane32_swap(y, y): {rows
  // (y0, y0, y0, y0)... i.e. the low half broadcast, the high half broadcast}
  const auto a = __builtin_amdgcn_permlane16_swap(p, p, false, false);
  const auto b = __builtin_amdgcn_permlane32_swap(a[0], a[0], false, false);
  const auto d = __builtin_amdgcn_permlane32_swap(a[1], a[1], false, false);
  o0 = b[0];
  o2 = b[1];
  o1 = d[0];
  o3 = d[1];
#else
  const int j4 = (int)(threadIdx.x & 15) * 4;
  o0 = (uint32_t)__builtin_amdgcn_ds_bpermute(j4, (int)p);
  o1 = (uint32_t)__builtin_amdgcn_ds_bpermute(j4 + 64, (int)p);
  o2 = (uint32_t)__builtin_amdgcn_ds_bpermute(j4 + 128, (int)p);
  o3 = (uint32_t)__builtin_amdgcn_ds_bpermute(j4 + 192, (int)p);
#endif
}
// one round: o_k = x_k y_k (row k's product)
__device__ __forceinline__ void mul4(const Ctx &c, uint32_t &o0, uint32_t &o1, uint32_t &o2,
                                     uint32_t &o3, uint32_t x0, uint32_t y0, uint32_t x1,
                                     uint32_t y1, uint32_t x2, uint32_t y2, uint32_t x3,
                                     uint32_t y3) {
  const uint32_t p = dfp::mul(sel(c, x0, x1, x2, x3), sel(c, y0, y1, y2, y3), c.t);
  gather(p, o0, o1, o2, o3);
}
// one round of dual products: o_k = x_k y_k + z_k w_k (one reduction, output < 1.0001 p)
__device__ __forceinline__ void mul4d(const Ctx &c, uint32_t &o0, uint32_t &o1, uint32_t &o2,
                                      uint32_t &o3, const uint32_t (&x)[4], const uint32_t (&y)[4],
                                      const uint32_t (&z)[4], const uint32_t (&w)[4]) {
  const uint32_t p = dfp::mul2(sel(c, x[0], x[1], x[2], x[3]), sel(c, y[0], y[1], y[2], y[3]),
                               sel(c, z[0], z[1], z[2], z[3]), sel(c, w[0], w[1], w[2], w[3]), c.t);
  gather(p, o0, o1, o2, o3);
}
// zero tests of four values (< 2^392): bit k set when value k = 0 mod p (one round)
__device__ __forceinline__ uint32_t zero4(const Ctx &c, uint32_t v0, uint32_t v1, uint32_t v2,
                                          uint32_t v3) {
  const bool z = dfp::is_zero(sel(c, v0, v1, v2, v3), c.t);
  const uint64_t m = __ballot(z);
  return (uint32_t)(m & 1) | (uint32_t)((m >> 15) & 2) | (uint32_t)((m >> 30) & 4) |
         (uint32_t)((m >> 45) & 8);
}

// ---- lane-local Fp
// The subtrahend of sub() is made opaque to the optimizer: otherwise it reassociates
// a + bias - ((x & M) + row_shr(c)) into (a + bias - (x & M)) - row_shr(c), which the DPP
// combiner turns into v_subrev_u32_dpp, measured wrong on MI355X (tools/ubench/w4_prim:
// the doubling and addition fail with the combine, pass without it).
__device__ __forceinline__ uint32_t opaque(uint32_t v) {
  asm volatile("" : "+v"(v));
  return v;
}
__device__ __forceinline__ uint32_t add(uint32_t a, uint32_t b) { return dfp::norm(a + b); }
template <int K>  // a + 2^K p - b
__device__ __forceinline__ uint32_t sub(const Ctx &c, uint32_t a, uint32_t b) {
  static_assert(K >= 1 && K <= 10, "bias table holds 2p .. 1024p");
  return dfp::norm(a + c.bias[K - 1] - opaque(b));
}
__device__ __forceinline__ uint32_t small(uint32_t a, uint32_t k) { return dfp::norm(a * k); }
// a / 2 mod p: the value's parity is limb 0's (higher limbs weigh 2^28); odd -> add p first
__device__ __forceinline__ uint32_t half(const Ctx &c, uint32_t a) {
  const uint32_t odd = dfp::bcast<0>(a) & 1u;
  const uint32_t x = odd ? a + dfp::K_P[c.t.j] : a;  // limbs < 2^29 + 2^10
  const uint32_t up = dfp::shl<1>(x);                  // limb j + 1 (0 past lane 15)
  return dfp::norm((x >> 1) + ((up & 1u) << 27));
}

// ---- Fp2 (c0 + c1 u, u^2 = -1)
struct f2 {
  uint32_t c0, c1;
};
__device__ __forceinline__ f2 add(const f2 &a, const f2 &b) { return {add(a.c0, b.c0), add(a.c1, b.c1)}; }
template <int K0, int K1>
__device__ __forceinline__ f2 sub(const Ctx &c, const f2 &a, const f2 &b) {
  return {sub<K0>(c, a.c0, b.c0), sub<K1>(c, a.c1, b.c1)};
}
__device__ __forceinline__ f2 small(const f2 &a, uint32_t k) { return {small(a.c0, k), small(a.c1, k)}; }
template <int K0, int K1>
__device__ __forceinline__ f2 neg(const Ctx &c, const f2 &a) {
  return {sub<K0>(c, 0u, a.c0), sub<K1>(c, 0u, a.c1)};
}
__device__ __forceinline__ f2 half(const Ctx &c, const f2 &a) { return {half(c, a.c0), half(c, a.c1)}; }
// Karatsuba recombination of t0 = a0 b0, t1 = a1 b1, t2 = (a0 + a1)(b0 + b1): (< 3, < 5)
__device__ __forceinline__ f2 kara(const Ctx &c, uint32_t t0, uint32_t t1, uint32_t t2) {
  return {sub<1>(c, t0, t1), sub<2>(c, t2, add(t0, t1))};
}
// squaring from s0 = (a0 + a1)(a0 - a1), s1 = a0 a1: (< 1.0001, < 2.0002)
__device__ __forceinline__ f2 sqr_of(uint32_t s0, uint32_t s1) { return {s0, add(s1, s1)}; }

// ---- points in row form
struct J {  // Jacobian (x = X/Z^2, y = Y/Z^3) or homogeneous (Miller T), Z = 0 is infinity
  f2 x, y, z;
};
struct A2 {
  f2 x, y;
};

// engine-form Fp2 words (x 2^384) -> row form: the repacked 28-bit limbs of lane j
__device__ __forceinline__ uint32_t repack(const fp &a, uint32_t j) {
  uint32_t v = 0;
#pragma unroll
  for (int i = 0; i < 14; i++) {
    const int bit = 28 * i, k = bit >> 5, sh = bit & 31;
    uint64_t pair = a.l[k];
    if (k + 1 < 12) pair |= (uint64_t)a.l[k + 1] << 32;
    const uint32_t limb = (uint32_t)(pair >> sh) & dfp::M28;
    v = j == (uint32_t)i ? limb : v;
  }
  return v;
}
// engine Jacobian point -> row form (2 rounds: 6 conversion products)
__device__ __forceinline__ void load(const Ctx &c, J &o, const g2j &p) {
  const uint32_t cin = dfp::konst(dfp::K_CIN);
  uint32_t v[6] = {repack(p.x.c0, c.t.j), repack(p.x.c1, c.t.j), repack(p.y.c0, c.t.j),
                   repack(p.y.c1, c.t.j), repack(p.z.c0, c.t.j), repack(p.z.c1, c.t.j)};
  mul4(c, o.x.c0, o.x.c1, o.y.c0, o.y.c1, v[0], cin, v[1], cin, v[2], cin, v[3], cin);
  uint32_t d0, d1;
  mul4(c, o.z.c0, o.z.c1, d0, d1, v[4], cin, v[5], cin, v[4], cin, v[5], cin);
}
__device__ __forceinline__ void load(const Ctx &c, A2 &o, const g2a &p) {
  const uint32_t cin = dfp::konst(dfp::K_CIN);
  mul4(c, o.x.c0, o.x.c1, o.y.c0, o.y.c1, repack(p.x.c0, c.t.j), cin, repack(p.x.c1, c.t.j), cin,
       repack(p.y.c0, c.t.j), cin, repack(p.y.c1, c.t.j), cin);
}
// four values -> canonical engine-form words at w0..w3 (one round; row k stores value k)
__device__ __forceinline__ void store4(const Ctx &c, uint32_t v0, uint32_t v1, uint32_t v2,
                                       uint32_t v3, uint32_t *w0, uint32_t *w1, uint32_t *w2,
                                       uint32_t *w3) {
  uint32_t *w = c.r == 0 ? w0 : (c.r == 1 ? w1 : (c.r == 2 ? w2 : w3));
  dfp::to_words(w, sel(c, v0, v1, v2, v3), c.t);
}

// row-form point -> canonical engine-form Jacobian words (two rounds)
__device__ __forceinline__ void store_jac(const Ctx &c, g2j *o, const J &p) {
  store4(c, p.x.c0, p.x.c1, p.y.c0, p.y.c1, o->x.c0.l, o->x.c1.l, o->y.c0.l, o->y.c1.l);
  const uint32_t w = dfp::word_of(sel(c, p.z.c0, p.z.c1, p.z.c0, p.z.c1), c.t);
  if (c.t.j < 12 && c.r == 0) o->z.c0.l[c.t.j] = w;
  if (c.t.j < 12 && c.r == 1) o->z.c1.l[c.t.j] = w;
}

// ---- G2 point formulas
// dbl-2009-l, inputs < 600 p; out X (< 33, < 66), Y (< 19, < 37), Z (< 6, < 10).  o may alias p.
#ifdef W4_NOINLINE
__device__ __noinline__
#else
__device__ __forceinline__
#endif
void dbl(const Ctx &c, J &o, const J &p) {
  // R1: A = X^2, B = Y^2
  uint32_t a0, ax, b0, bx;
  mul4(c, a0, ax, b0, bx, add(p.x.c0, p.x.c1), sub<10>(c, p.x.c0, p.x.c1), p.x.c0, p.x.c1,
       add(p.y.c0, p.y.c1), sub<10>(c, p.y.c0, p.y.c1), p.y.c0, p.y.c1);
  const f2 A = sqr_of(a0, ax), B = sqr_of(b0, bx);  // (< 1.0001, < 2.0002)
  const f2 E = small(A, 3);                           // (< 3.0003, < 6.0006)
  // R2: C = B^2, F = E^2
  uint32_t c0, cx, f0, fx;
  mul4(c, c0, cx, f0, fx, add(B.c0, B.c1), sub<2>(c, B.c0, B.c1), B.c0, B.c1, add(E.c0, E.c1),
       sub<3>(c, E.c0, E.c1), E.c0, E.c1);
  const f2 C = sqr_of(c0, cx), F = sqr_of(f0, fx);
  // R3: (X + B)^2, y0 z0, y1 z1
  const f2 t = add(p.x, B);
  uint32_t g0, gx, yz0, yz1;
  mul4(c, g0, gx, yz0, yz1, add(t.c0, t.c1), sub<10>(c, t.c0, t.c1), t.c0, t.c1, p.y.c0, p.z.c0,
       p.y.c1, p.z.c1);
  const f2 XB2 = sqr_of(g0, gx);
  // D = 2((X + B)^2 - A - C): (< 10.001, < 20.002)
  const f2 D = small(sub<2, 3>(c, XB2, add(A, C)), 2);
  const f2 X3 = sub<5, 6>(c, F, small(D, 2));  // (< 33.001, < 66.001)
  const f2 u = sub<6, 7>(c, D, X3);            // (< 74.002, < 148.01)
  // R4: E (D - X3) and (y0 + y1)(z0 + z1)
  uint32_t m0, m1, m2, yz2;
  mul4(c, m0, m1, m2, yz2, E.c0, u.c0, E.c1, u.c1, add(E.c0, E.c1), add(u.c0, u.c1),
       add(p.y.c0, p.y.c1), add(p.z.c0, p.z.c1));
  const f2 Eu = kara(c, m0, m1, m2);
  const f2 YZ = kara(c, yz0, yz1, yz2);
  o.x = X3;
  o.y = sub<4, 5>(c, Eu, small(C, 8));  // (< 19.001, < 37.001)
  o.z = small(YZ, 2);                   // (< 6.0002, < 10.001)
}

__device__ __forceinline__ void set_inf(const Ctx &c, J &o) {
  o.x = {c.one, 0u};
  o.y = {c.one, 0u};
  o.z = {0u, 0u};
}
// Z = 0 mod p (one round)
__device__ __forceinline__ bool is_inf(const Ctx &c, const J &p) {
  return zero4(c, p.z.c0, p.z.c1, p.z.c0, p.z.c1) == 0xf;
}

// add-2007-bl, r = a + b, inputs < 600 p; out X (< 17.001, < 18.001), Y (< 11.001, < 21.001),
// Z (< 3.0001, < 5.0001), or a copy of an input (a = inf / b = inf), or dbl(b) (a = b), or
// infinity (a = -b) -- jac_add's cases (bls_curve.h).  o may alias a or b.
__device__ __forceinline__ void add(const Ctx &c, J &o, const J &a, const J &b) {
  const uint32_t zf = zero4(c, a.z.c0, a.z.c1, b.z.c0, b.z.c1);
  if ((zf & 0xc) == 0xc) {  // b = inf
    o = a;
    return;
  }
  if ((zf & 0x3) == 0x3) {  // a = inf
    o = b;
    return;
  }
  // R1: Z1^2, Z2^2
  uint32_t p0, px, q0, qx;
  mul4(c, p0, px, q0, qx, add(a.z.c0, a.z.c1), sub<10>(c, a.z.c0, a.z.c1), a.z.c0, a.z.c1,
       add(b.z.c0, b.z.c1), sub<10>(c, b.z.c0, b.z.c1), b.z.c0, b.z.c1);
  const f2 Z1Z1 = sqr_of(p0, px), Z2Z2 = sqr_of(q0, qx);
  // R2: U1 = X1 Z2Z2, y10 z20
  uint32_t m0, m1, m2, s0;
  mul4(c, m0, m1, m2, s0, a.x.c0, Z2Z2.c0, a.x.c1, Z2Z2.c1, add(a.x.c0, a.x.c1),
       add(Z2Z2.c0, Z2Z2.c1), a.y.c0, b.z.c0);
  const f2 U1 = kara(c, m0, m1, m2);
  // R3: U2 = X2 Z1Z1, y11 z21
  uint32_t s1;
  mul4(c, m0, m1, m2, s1, b.x.c0, Z1Z1.c0, b.x.c1, Z1Z1.c1, add(b.x.c0, b.x.c1),
       add(Z1Z1.c0, Z1Z1.c1), a.y.c1, b.z.c1);
  const f2 U2 = kara(c, m0, m1, m2);
  // R4: (y10 + y11)(z20 + z21); Y2 Z1
  uint32_t s2, n0, n1, n2;
  mul4(c, s2, n0, n1, n2, add(a.y.c0, a.y.c1), add(b.z.c0, b.z.c1), b.y.c0, a.z.c0, b.y.c1, a.z.c1,
       add(b.y.c0, b.y.c1), add(a.z.c0, a.z.c1));
  const f2 Y1Z2 = kara(c, s0, s1, s2), Y2Z1 = kara(c, n0, n1, n2);
  const f2 zs = add(a.z, b.z);
  // R5: S1 = Y1Z2 Z2Z2, (Z1 + Z2)^2 [0]
  uint32_t w0, wx;
  mul4(c, m0, m1, m2, w0, Y1Z2.c0, Z2Z2.c0, Y1Z2.c1, Z2Z2.c1, add(Y1Z2.c0, Y1Z2.c1),
       add(Z2Z2.c0, Z2Z2.c1), add(zs.c0, zs.c1), sub<10>(c, zs.c0, zs.c1));
  const f2 S1 = kara(c, m0, m1, m2);
  // R6: S2 = Y2Z1 Z1Z1, (Z1 + Z2)^2 [1]
  mul4(c, m0, m1, m2, wx, Y2Z1.c0, Z1Z1.c0, Y2Z1.c1, Z1Z1.c1, add(Y2Z1.c0, Y2Z1.c1),
       add(Z1Z1.c0, Z1Z1.c1), zs.c0, zs.c1);
  const f2 S2 = kara(c, m0, m1, m2);
  const f2 H = sub<2, 3>(c, U2, U1);                    // (< 7.0001, < 10.001)
  const f2 rr = small(sub<2, 3>(c, S2, S1), 2);         // (< 14.001, < 20.002)
  const f2 ZZ = sub<2, 3>(c, sqr_of(w0, wx), add(Z1Z1, Z2Z2));  // 2 Z1 Z2 (< 5.0003, < 10.001)
  const uint32_t hf = zero4(c, H.c0, H.c1, rr.c0, rr.c1);
  if ((hf & 3) == 3) {
    if ((hf & 0xc) == 0xc) {
      dbl(c, o, b);
    } else {
      set_inf(c, o);
    }
    return;
  }
  // R7: I = (2H)^2, rr^2
  const f2 h2 = small(H, 2);  // (< 14.001, < 20.002)
  uint32_t i0, ix, r0, rx;
  mul4(c, i0, ix, r0, rx, add(h2.c0, h2.c1), sub<5>(c, h2.c0, h2.c1), h2.c0, h2.c1,
       add(rr.c0, rr.c1), sub<5>(c, rr.c0, rr.c1), rr.c0, rr.c1);
  const f2 I = sqr_of(i0, ix), R2 = sqr_of(r0, rx);
  // R8: J = H I, V = U1 I [0]
  uint32_t v0;
  mul4(c, m0, m1, m2, v0, H.c0, I.c0, H.c1, I.c1, add(H.c0, H.c1), add(I.c0, I.c1), U1.c0, I.c0);
  const f2 Jv = kara(c, m0, m1, m2);
  // R9: V [1, 2], ZZ H [0, 1]
  uint32_t v1, v2, z0, z1;
  mul4(c, v1, v2, z0, z1, U1.c1, I.c1, add(U1.c0, U1.c1), add(I.c0, I.c1), ZZ.c0, H.c0, ZZ.c1, H.c1);
  const f2 V = kara(c, v0, v1, v2);
  const f2 X3 = sub<4, 4>(c, R2, add(Jv, small(V, 2)));  // (< 17.001, < 18.001)
  const f2 wv = sub<5, 5>(c, V, X3);                     // (< 35.002, < 37.002)
  // R10: ZZ H [2], S1 J
  uint32_t z2;
  mul4(c, z2, m0, m1, m2, add(ZZ.c0, ZZ.c1), add(H.c0, H.c1), S1.c0, Jv.c0, S1.c1, Jv.c1,
       add(S1.c0, S1.c1), add(Jv.c0, Jv.c1));
  const f2 S1J = kara(c, m0, m1, m2);
  const f2 Z3 = kara(c, z0, z1, z2);
  // R11: rr (V - X3)
  uint32_t d;
  mul4(c, m0, m1, m2, d, rr.c0, wv.c0, rr.c1, wv.c1, add(rr.c0, rr.c1), add(wv.c0, wv.c1), rr.c0,
       wv.c0);
  const f2 rw = kara(c, m0, m1, m2);
  o.x = X3;
  o.y = sub<3, 4>(c, rw, small(S1J, 2));  // (< 11.001, < 21.001)
  o.z = Z3;
}

// madd-2007-bl, r = a + b for an affine b (not infinity), a.x < 120 p, a.y < 60 p, a.z < 600 p
// (dbl / madd outputs): jac_add_aff's cases
// (bls_curve.h: a = inf -> b; a = b -> dbl(b); a = -b -> inf).  Eight rounds + a zero test;
// out X (< 17.001, < 18.001), Y (< 11.001, < 21.001), Z (< 5.0003, < 10.001).  o may alias a.
__device__ __forceinline__ void madd(const Ctx &c, J &o, const J &a, const A2 &b) {
  const uint32_t zs = add(a.z.c0, a.z.c1);
  // R1: Z1^2, y20 z10, y21 z11
  uint32_t p0, px, s0, s1;
  mul4(c, p0, px, s0, s1, zs, sub<10>(c, a.z.c0, a.z.c1), a.z.c0, a.z.c1, b.y.c0, a.z.c0, b.y.c1,
       a.z.c1);
  const f2 Z1Z1 = sqr_of(p0, px);
  // R2: Y2 Z1 [2], U2 = X2 Z1Z1
  uint32_t s2, m0, m1, m2;
  mul4(c, s2, m0, m1, m2, add(b.y.c0, b.y.c1), zs, b.x.c0, Z1Z1.c0, b.x.c1, Z1Z1.c1,
       add(b.x.c0, b.x.c1), add(Z1Z1.c0, Z1Z1.c1));
  const f2 Y2Z1 = kara(c, s0, s1, s2), U2 = kara(c, m0, m1, m2);
  // R3: S2 = Y2Z1 Z1Z1
  uint32_t d;
  mul4(c, m0, m1, m2, d, Y2Z1.c0, Z1Z1.c0, Y2Z1.c1, Z1Z1.c1, add(Y2Z1.c0, Y2Z1.c1),
       add(Z1Z1.c0, Z1Z1.c1), Y2Z1.c0, Z1Z1.c0);
  const f2 S2 = kara(c, m0, m1, m2);
  const f2 H = sub<7, 7>(c, U2, a.x);             // (< 131, < 133)
  const f2 rr = small(sub<6, 6>(c, S2, a.y), 2);  // (< 134, < 138)
  const uint32_t zf = zero4(c, H.c0, H.c1, a.z.c0, a.z.c1);
  if ((zf & 0xc) == 0xc) {  // a = inf
    o.x = b.x;
    o.y = b.y;
    o.z = {c.one, 0u};
    return;
  }
  if ((zf & 3) == 3) {
    const uint32_t rf = zero4(c, rr.c0, rr.c1, rr.c0, rr.c1);
    if (rf == 0xf) {
      J bj;
      bj.x = b.x;
      bj.y = b.y;
      bj.z = {c.one, 0u};
      dbl(c, o, bj);
    } else {
      set_inf(c, o);
    }
    return;
  }
  // R4: HH = H^2, rr^2
  uint32_t h0, hx, r0, rx;
  mul4(c, h0, hx, r0, rx, add(H.c0, H.c1), sub<8>(c, H.c0, H.c1), H.c0, H.c1, add(rr.c0, rr.c1),
       sub<8>(c, rr.c0, rr.c1), rr.c0, rr.c1);
  const f2 HH = sqr_of(h0, hx), R2 = sqr_of(r0, rx);
  const f2 I = small(HH, 4);  // (< 4.0004, < 8.0008)
  // R5: J = H I, V = X1 I [0]
  uint32_t v0;
  mul4(c, m0, m1, m2, v0, H.c0, I.c0, H.c1, I.c1, add(H.c0, H.c1), add(I.c0, I.c1), a.x.c0, I.c0);
  const f2 Jv = kara(c, m0, m1, m2);
  // R6: V [1, 2], (Z1 + H)^2
  const f2 zh = add(a.z, H);  // < 743
  uint32_t v1, v2, w0, wx;
  mul4(c, v1, v2, w0, wx, a.x.c1, I.c1, add(a.x.c0, a.x.c1), add(I.c0, I.c1), add(zh.c0, zh.c1),
       sub<10>(c, zh.c0, zh.c1), zh.c0, zh.c1);
  const f2 V = kara(c, v0, v1, v2);
  const f2 X3 = sub<4, 4>(c, R2, add(Jv, small(V, 2)));  // (< 17.001, < 18.001)
  const f2 wv = sub<5, 5>(c, V, X3);
  // R7: Y1 J, rr (V - X3) [0]
  uint32_t q0, q1, q2, k0;
  mul4(c, q0, q1, q2, k0, a.y.c0, Jv.c0, a.y.c1, Jv.c1, add(a.y.c0, a.y.c1), add(Jv.c0, Jv.c1),
       rr.c0, wv.c0);
  // R8: rr (V - X3) [1, 2]
  uint32_t k1, k2, d1;
  mul4(c, k1, k2, d, d1, rr.c1, wv.c1, add(rr.c0, rr.c1), add(wv.c0, wv.c1), rr.c1, wv.c1, rr.c1,
       wv.c1);
  o.x = X3;
  o.y = sub<3, 4>(c, kara(c, k0, k1, k2), small(kara(c, q0, q1, q2), 2));  // (< 11.001, < 21.001)
  o.z = sub<2, 3>(c, sqr_of(w0, wx), add(Z1Z1, HH));                       // (< 5.0003, < 10.001)
}

// psi(P) = (conj(X) cx, conj(Y) cy, conj(Z)), cx = PSI_CX1 u: one dual-product round.
// out X, Y < 1.0001; Z = (z0, 2^KZ p - z1).  o may alias p.
template <int KZ>
__device__ __forceinline__ void psi(const Ctx &c, J &o, const J &p) {
  const uint32_t cx = dfp::konst(dfp::K_PSI_CX1), cy0 = dfp::konst(dfp::K_PSI_CY0),
                 cy1 = dfp::konst(dfp::K_PSI_CY1);
  const uint32_t ny1 = sub<10>(c, 0u, p.y.c1);
  // (x0 - x1 u)(cx u) = x1 cx + x0 cx u; (y0 - y1 u)(cy0 + cy1 u) = (y0 cy0 + y1 cy1) + (y0 cy1 - y1 cy0) u
  const uint32_t X[4] = {p.x.c1, p.x.c0, p.y.c0, p.y.c0}, Y[4] = {cx, cx, cy0, cy1};
  const uint32_t Z[4] = {0u, 0u, p.y.c1, ny1}, W[4] = {0u, 0u, cy1, cy0};
  f2 x, y;
  mul4d(c, x.c0, x.c1, y.c0, y.c1, X, Y, Z, W);
  o.x = x;
  o.y = y;
  o.z = {p.z.c0, sub<KZ>(c, 0u, p.z.c1)};
}
// psi^2(P) = (X PSI2_CX, Y PSI2_CY, Z) with Fp constants: one round; out X, Y < 1.0001
__device__ __forceinline__ void psi2(const Ctx &c, J &o, const J &p) {
  const uint32_t kx = dfp::konst(dfp::K_PSI2_CX), ky = dfp::konst(dfp::K_PSI2_CY);
  mul4(c, o.x.c0, o.x.c1, o.y.c0, o.y.c1, p.x.c0, kx, p.x.c1, kx, p.y.c0, ky, p.y.c1, ky);
  o.z = p.z;
}
template <int K0, int K1>
__device__ __forceinline__ void negy(const Ctx &c, J &o, const J &p) {
  o.x = p.x;
  o.y = neg<K0, K1>(c, p.y);
  o.z = p.z;
}

// [|x|]P (|x| = 0xd201000000010000): 63 doublings, 5 additions of P.  r must not alias p.
__device__ __forceinline__ void mul_by_xabs(const Ctx &c, J &r, const J &p) {
  r = p;
  for (int i = 62; i >= 0; i--) {
    dbl(c, r, r);
    if ((dfp::X_ABS >> i) & 1) add(c, r, r, p);
  }
}

// h_eff P (clear_cofactor_g2, bls_hash.h: Budroni-Pintore), the lane code's sequence.
// Input coordinates < 64 p.  r must not alias p.
__device__ __forceinline__ void clear_cofactor(const Ctx &c, J &r, const J &p) {
  J t1, t2, t3;
  mul_by_xabs(c, t1, p);
  negy<6, 6>(c, t1, t1);  // t1 = [x]P          y < 64
  psi<7>(c, t2, p);
  add(c, t2, t2, t1);     // t1 + psi(P)
  mul_by_xabs(c, t3, t2);
  negy<6, 6>(c, t3, t3);  // t3 = [x](t1 + psi(P))
  negy<7, 7>(c, t1, t1);  // y < 128
  add(c, t3, t3, t1);     // - t1
  dbl(c, t1, p);
  psi2(c, t1, t1);
  add(c, t3, t3, t1);     // + psi^2(2P)
  psi<7>(c, t1, p);
  negy<1, 1>(c, t1, t1);  // psi's y < 1.0001
  add(c, t3, t3, t1);     // - psi(P)
  negy<7, 7>(c, t1, p);
  add(c, r, t3, t1);      // - P
}

// ---- Miller-loop steps (bls_pairing.h line_dbl / line_add_aff: the same values mod p)
// Doubling step on a homogeneous T (inputs < 600 p): L0 = 3b'Z^2 - Y^2, L2 = 3X^2, L3 = -2YZ;
// out T (< 3, < 5), (< 5.0004, < 10.001), (< 3, < 5).  Six rounds.
__device__ __forceinline__ void line_dbl(const Ctx &c, J &T, f2 &L0, f2 &L2, f2 &L3) {
  // R1: B = Y^2, C = Z^2
  uint32_t b0, bx, c0, cx;
  mul4(c, b0, bx, c0, cx, add(T.y.c0, T.y.c1), sub<10>(c, T.y.c0, T.y.c1), T.y.c0, T.y.c1,
       add(T.z.c0, T.z.c1), sub<10>(c, T.z.c0, T.z.c1), T.z.c0, T.z.c1);
  const f2 B = sqr_of(b0, bx), C = sqr_of(c0, cx);
  const f2 xiC = {sub<2>(c, C.c0, C.c1), add(C.c0, C.c1)};  // (1 + u) C
  const f2 E = small(xiC, 12);                               // 3 b' C (< 60.004, < 36.004)
  const f2 F = small(E, 3);                                  // (< 180.02, < 108.02)
  const f2 G = half(c, add(B, F));                           // (< 91.01, < 55.51)
  L0 = sub<1, 2>(c, E, B);
  // R2: X Y (3), X^2 [0]
  const f2 xs = {add(T.x.c0, T.x.c1), sub<10>(c, T.x.c0, T.x.c1)};
  uint32_t m0, m1, m2, s0;
  mul4(c, m0, m1, m2, s0, T.x.c0, T.y.c0, T.x.c1, T.y.c1, xs.c0, add(T.y.c0, T.y.c1), xs.c0, xs.c1);
  const f2 A = half(c, kara(c, m0, m1, m2));  // XY / 2 (< 2.0001, < 3.0001)
  // R3: X^2 [1], (Y + Z)^2, E^2 [0]
  const f2 t = add(T.y, T.z);
  uint32_t sx, h0, hx, e0;
  mul4(c, sx, h0, hx, e0, T.x.c0, T.x.c1, add(t.c0, t.c1), sub<10>(c, t.c0, t.c1), t.c0, t.c1,
       add(E.c0, E.c1), sub<6>(c, E.c0, E.c1));
  L2 = small(sqr_of(s0, sx), 3);
  const f2 H = sub<2, 3>(c, sqr_of(h0, hx), add(B, C));  // 2YZ (< 5.0003, < 10.001)
  L3 = neg<3, 4>(c, H);
  const f2 w = sub<8, 7>(c, B, F);  // B - F (< 257.01, < 130.01)
  // R4: E^2 [1], G^2, A (B - F) [0]
  uint32_t ex, g0, gx, a0;
  mul4(c, ex, g0, gx, a0, E.c0, E.c1, add(G.c0, G.c1), sub<6>(c, G.c0, G.c1), G.c0, G.c1, A.c0, w.c0);
  // R5: A (B - F) [1, 2], B H [0, 1]
  uint32_t a1, a2, z0, z1;
  mul4(c, a1, a2, z0, z1, A.c1, w.c1, add(A.c0, A.c1), add(w.c0, w.c1), B.c0, H.c0, B.c1, H.c1);
  // R6: B H [2]
  uint32_t z2, d0, d1, d2;
  const uint32_t bs = add(B.c0, B.c1), hs = add(H.c0, H.c1);
  mul4(c, z2, d0, d1, d2, bs, hs, bs, hs, bs, hs, bs, hs);
  T.x = kara(c, a0, a1, a2);
  T.z = kara(c, z0, z1, z2);
  T.y = sub<2, 3>(c, sqr_of(g0, gx), small(sqr_of(e0, ex), 3));  // G^2 - 3E^2
}

// Addition step T + Q for an affine Q (inputs T < 64 p, Q < 2 p):
//   theta = Y1 - y2 Z1, lambda = X1 - x2 Z1;  L0 = theta x2 - lambda y2, L2 = -theta, L3 = lambda;
//   with nv = lambda^3: X3 = -lambda A, Y3 = nv Y1 - theta (R - A), Z3 = -nv Z1,
//   R = lambda^2 X1, A = theta^2 Z1 + nv - 2R.  Out T (< 4, < 8), (< 7, < 13), (< 4, < 8).
__device__ __forceinline__ void line_add_aff(const Ctx &c, J &T, const A2 &Q, f2 &L0, f2 &L2,
                                             f2 &L3) {
  const uint32_t zs = add(T.z.c0, T.z.c1);
  // R1: y2 Z1, x20 z10
  uint32_t m0, m1, m2, x0;
  mul4(c, m0, m1, m2, x0, Q.y.c0, T.z.c0, Q.y.c1, T.z.c1, add(Q.y.c0, Q.y.c1), zs, Q.x.c0, T.z.c0);
  const f2 th = sub<2, 3>(c, T.y, kara(c, m0, m1, m2));  // (< 68, < 72)
  // R2: x2 Z1 [1, 2], theta^2
  uint32_t x1, x2, u0, ux;
  mul4(c, x1, x2, u0, ux, Q.x.c1, T.z.c1, add(Q.x.c0, Q.x.c1), zs, add(th.c0, th.c1),
       sub<7>(c, th.c0, th.c1), th.c0, th.c1);
  const f2 la = sub<2, 3>(c, T.x, kara(c, x0, x1, x2));
  const f2 uu = sqr_of(u0, ux);
  // R3: lambda^2, theta x2 [0, 1]
  uint32_t v0, vx, p0, p1;
  mul4(c, v0, vx, p0, p1, add(la.c0, la.c1), sub<7>(c, la.c0, la.c1), la.c0, la.c1, th.c0, Q.x.c0,
       th.c1, Q.x.c1);
  const f2 vv = sqr_of(v0, vx);
  // R4: theta x2 [2], lambda y2
  uint32_t p2, q0, q1, q2;
  mul4(c, p2, q0, q1, q2, add(th.c0, th.c1), add(Q.x.c0, Q.x.c1), la.c0, Q.y.c0, la.c1, Q.y.c1,
       add(la.c0, la.c1), add(Q.y.c0, Q.y.c1));
  L0 = sub<2, 3>(c, kara(c, p0, p1, p2), kara(c, q0, q1, q2));
  L2 = neg<7, 7>(c, th);
  L3 = la;
  // R5: nv = vv lambda, R = vv X1 [0]
  uint32_t r0;
  mul4(c, m0, m1, m2, r0, vv.c0, la.c0, vv.c1, la.c1, add(vv.c0, vv.c1), add(la.c0, la.c1), vv.c0,
       T.x.c0);
  const f2 nv = kara(c, m0, m1, m2);
  // R6: R [1, 2], uu Z1 [0, 1]
  uint32_t r1, r2, w0, w1;
  mul4(c, r1, r2, w0, w1, vv.c1, T.x.c1, add(vv.c0, vv.c1), add(T.x.c0, T.x.c1), uu.c0, T.z.c0,
       uu.c1, T.z.c1);
  const f2 R = kara(c, r0, r1, r2);
  // R7: uu Z1 [2], nv Y1
  uint32_t w2, y0, y1, y2;
  mul4(c, w2, y0, y1, y2, add(uu.c0, uu.c1), zs, nv.c0, T.y.c0, nv.c1, T.y.c1, add(nv.c0, nv.c1),
       add(T.y.c0, T.y.c1));
  const f2 A = sub<3, 4>(c, add(kara(c, w0, w1, w2), nv), small(R, 2));  // (< 14, < 26)
  const f2 rma = sub<5, 5>(c, R, A);
  // R8: nv Z1, lambda A [0]
  uint32_t z0, z1, z2, l0;
  mul4(c, z0, z1, z2, l0, nv.c0, T.z.c0, nv.c1, T.z.c1, add(nv.c0, nv.c1), zs, la.c0, A.c0);
  // R9: lambda A [1, 2], theta (R - A) [0, 1]
  uint32_t l1, l2, k0, k1;
  mul4(c, l1, l2, k0, k1, la.c1, A.c1, add(la.c0, la.c1), add(A.c0, A.c1), th.c0, rma.c0, th.c1,
       rma.c1);
  // R10: theta (R - A) [2]
  uint32_t k2, d0, d1, d2;
  const uint32_t ts = add(th.c0, th.c1), rs = add(rma.c0, rma.c1);
  mul4(c, k2, d0, d1, d2, ts, rs, ts, rs, ts, rs, ts, rs);
  T.x = neg<2, 3>(c, kara(c, l0, l1, l2));
  T.y = sub<2, 3>(c, kara(c, y0, y1, y2), kara(c, k0, k1, k2));
  T.z = neg<2, 3>(c, kara(c, z0, z1, z2));
}

// Addition step T + Q for a homogeneous Q = (Xq, Yq, Zq) (T < 64 p, Q < 64 p): the general
// add-1998-cmo-2 update and the line through T and Q scaled by Zq^2 (an Fp2 factor, which the
// final exponentiation removes):
//   th = Y1 Zq - Yq Z1, la = X1 Zq - Xq Z1;  L0 = th Xq - la Yq, L2 = -th Zq, L3 = la Zq;
//   nv = la^3, R = la^2 X1 Zq, A = th^2 Z1 Zq + nv - 2R:
//   X3 = -la A, Y3 = nv Y1 Zq - th (R - A), Z3 = -nv Z1 Zq.
// 13 rounds; out T (< 4, < 8), (< 7, < 13), (< 4, < 8).
__device__ __forceinline__ void line_add_proj(const Ctx &c, J &T, const J &Q, f2 &L0, f2 &L2,
                                              f2 &L3) {
  const uint32_t zqs = add(Q.z.c0, Q.z.c1), z1s = add(T.z.c0, T.z.c1);
  // R1: Y1 Zq, Yq Z1 [0]
  uint32_t a0, a1, a2, b0;
  mul4(c, a0, a1, a2, b0, T.y.c0, Q.z.c0, T.y.c1, Q.z.c1, add(T.y.c0, T.y.c1), zqs, Q.y.c0, T.z.c0);
  // R2: Yq Z1 [1, 2], X1 Zq [0, 1]
  uint32_t b1, b2, e0, e1;
  mul4(c, b1, b2, e0, e1, Q.y.c1, T.z.c1, add(Q.y.c0, Q.y.c1), z1s, T.x.c0, Q.z.c0, T.x.c1, Q.z.c1);
  // R3: X1 Zq [2], Xq Z1
  uint32_t e2, g0, g1, g2;
  mul4(c, e2, g0, g1, g2, add(T.x.c0, T.x.c1), zqs, Q.x.c0, T.z.c0, Q.x.c1, T.z.c1,
       add(Q.x.c0, Q.x.c1), z1s);
  const f2 Y1Zq = kara(c, a0, a1, a2), X1Zq = kara(c, e0, e1, e2);
  const f2 th = sub<2, 3>(c, Y1Zq, kara(c, b0, b1, b2));  // (< 7, < 13)
  const f2 la = sub<2, 3>(c, X1Zq, kara(c, g0, g1, g2));
  // R4: th^2, la^2
  uint32_t u0, ux, v0, vx;
  mul4(c, u0, ux, v0, vx, add(th.c0, th.c1), sub<4>(c, th.c0, th.c1), th.c0, th.c1,
       add(la.c0, la.c1), sub<4>(c, la.c0, la.c1), la.c0, la.c1);
  const f2 uu = sqr_of(u0, ux), vv = sqr_of(v0, vx);
  const uint32_t ths = add(th.c0, th.c1), las = add(la.c0, la.c1);
  // R5: th Xq, Z1 Zq [0]
  uint32_t p0, p1, p2, z0;
  mul4(c, p0, p1, p2, z0, th.c0, Q.x.c0, th.c1, Q.x.c1, ths, add(Q.x.c0, Q.x.c1), T.z.c0, Q.z.c0);
  // R6: la Yq, Z1 Zq [1]
  uint32_t q0, q1, q2, z1;
  mul4(c, q0, q1, q2, z1, la.c0, Q.y.c0, la.c1, Q.y.c1, las, add(Q.y.c0, Q.y.c1), T.z.c1, Q.z.c1);
  L0 = sub<2, 3>(c, kara(c, p0, p1, p2), kara(c, q0, q1, q2));
  // R7: th Zq, Z1 Zq [2]
  uint32_t r0, r1, r2, z2;
  mul4(c, r0, r1, r2, z2, th.c0, Q.z.c0, th.c1, Q.z.c1, ths, zqs, z1s, zqs);
  L2 = neg<2, 3>(c, kara(c, r0, r1, r2));
  const f2 Z1Zq = kara(c, z0, z1, z2);
  // R8: la Zq, nv = vv la [0]
  uint32_t s0, s1, s2, n0;
  mul4(c, s0, s1, s2, n0, la.c0, Q.z.c0, la.c1, Q.z.c1, las, zqs, vv.c0, la.c0);
  L3 = kara(c, s0, s1, s2);
  // R9: nv [1, 2], R = vv X1Zq [0, 1]
  uint32_t n1, n2, w0, w1;
  mul4(c, n1, n2, w0, w1, vv.c1, la.c1, add(vv.c0, vv.c1), las, vv.c0, X1Zq.c0, vv.c1, X1Zq.c1);
  const f2 nv = kara(c, n0, n1, n2);
  // R10: R [2], uu Z1Zq
  uint32_t w2, m0, m1, m2;
  mul4(c, w2, m0, m1, m2, add(vv.c0, vv.c1), add(X1Zq.c0, X1Zq.c1), uu.c0, Z1Zq.c0, uu.c1, Z1Zq.c1,
       add(uu.c0, uu.c1), add(Z1Zq.c0, Z1Zq.c1));
  const f2 R = kara(c, w0, w1, w2);
  const f2 A = sub<3, 4>(c, add(kara(c, m0, m1, m2), nv), small(R, 2));  // (< 14, < 26)
  const f2 rma = sub<5, 5>(c, R, A);
  // R11: la A, nv Y1Zq [0]
  uint32_t l0, l1, l2, y0;
  mul4(c, l0, l1, l2, y0, la.c0, A.c0, la.c1, A.c1, las, add(A.c0, A.c1), nv.c0, Y1Zq.c0);
  // R12: nv Y1Zq [1, 2], th (R - A) [0, 1]
  uint32_t y1, y2, k0, k1;
  mul4(c, y1, y2, k0, k1, nv.c1, Y1Zq.c1, add(nv.c0, nv.c1), add(Y1Zq.c0, Y1Zq.c1), th.c0, rma.c0,
       th.c1, rma.c1);
  // R13: th (R - A) [2], nv Z1Zq
  uint32_t k2, x0, x1, x2;
  mul4(c, k2, x0, x1, x2, ths, add(rma.c0, rma.c1), nv.c0, Z1Zq.c0, nv.c1, Z1Zq.c1,
       add(nv.c0, nv.c1), add(Z1Zq.c0, Z1Zq.c1));
  T.x = neg<2, 3>(c, kara(c, l0, l1, l2));
  T.y = sub<2, 3>(c, kara(c, y0, y1, y2), kara(c, k0, k1, k2));
  T.z = neg<2, 3>(c, kara(c, x0, x1, x2));
}
// Jacobian (X, Y, Z) -> homogeneous (X Z, Y, Z^3) of the same point (two rounds); out < 5 p
__device__ __forceinline__ void jac_to_hom(const Ctx &c, J &o, const J &p) {
  const uint32_t zs = add(p.z.c0, p.z.c1);
  uint32_t s0, sx, m0, m1;
  mul4(c, s0, sx, m0, m1, zs, sub<10>(c, p.z.c0, p.z.c1), p.z.c0, p.z.c1, p.x.c0, p.z.c0, p.x.c1,
       p.z.c1);
  const f2 Z2 = sqr_of(s0, sx);
  uint32_t m2, t0, t1, t2;
  mul4(c, m2, t0, t1, t2, add(p.x.c0, p.x.c1), zs, Z2.c0, p.z.c0, Z2.c1, p.z.c1,
       add(Z2.c0, Z2.c1), zs);
  o.x = kara(c, m0, m1, m2);
  o.y = p.y;
  o.z = kara(c, t0, t1, t2);
}

// ---- G1 (E: y^2 = x^3 + 4 over Fp) on the same rows: the random-scalar products r pk of the
// latency regime.  Jacobian over Fp; out bounds in units of p.
struct J1 {
  uint32_t x, y, z;
};
// dbl-2009-l, inputs < 600 p: 3 rounds; out X < 33.001, Y < 17.001, Z < 2.0002.  o may alias p.
__device__ __forceinline__ void dbl1(const Ctx &c, J1 &o, const J1 &p) {
  uint32_t A, B, yz, d;
  mul4(c, A, B, yz, d, p.x, p.x, p.y, p.y, p.y, p.z, p.x, p.x);
  const uint32_t E = small(A, 3), t = add(p.x, B);
  uint32_t C, T2, F;
  mul4(c, C, T2, F, d, B, B, t, t, E, E, E, E);
  const uint32_t D = small(sub<2>(c, T2, add(A, C)), 2);  // < 10.001
  const uint32_t X3 = sub<5>(c, F, small(D, 2));           // < 33.001
  const uint32_t u = sub<6>(c, D, X3);                     // < 74.002
  uint32_t eu, d1, d2;
  mul4(c, eu, d, d1, d2, E, u, E, u, E, u, E, u);
  o.x = X3;
  o.y = sub<4>(c, eu, small(C, 8));  // < 17.001
  o.z = small(yz, 2);                // < 2.0002
}
// madd-2007-bl, r = a + (x2, y2) (affine, not infinity), a.x < 120 p, a.y < 60 p (dbl1 / madd1
// outputs): 5 rounds + a zero test, jac_add_aff's cases; out X < 5.0004, Y < 5.0002, Z < 5.0003
__device__ __forceinline__ void madd1(const Ctx &c, J1 &o, const J1 &a, uint32_t x2, uint32_t y2) {
  uint32_t zz, yz, d, d1;
  mul4(c, zz, yz, d, d1, a.z, a.z, y2, a.z, a.z, a.z, a.z, a.z);
  uint32_t U2, S2;
  mul4(c, U2, S2, d, d1, x2, zz, yz, zz, x2, zz, x2, zz);
  const uint32_t H = sub<7>(c, U2, a.x);              // < 129
  const uint32_t rr = small(sub<6>(c, S2, a.y), 2);   // < 130
  const uint32_t zf = zero4(c, H, rr, a.z, a.z);
  if ((zf & 0xc) == 0xc) {  // a = inf
    o.x = x2;
    o.y = y2;
    o.z = c.one;
    return;
  }
  if (zf & 1) {
    if (zf & 2) {
      J1 bj{x2, y2, c.one};
      dbl1(c, o, bj);
    } else {
      o.x = c.one;
      o.y = c.one;
      o.z = 0u;
    }
    return;
  }
  const uint32_t zh = add(a.z, H);
  uint32_t HH, R2, ZH2;
  mul4(c, HH, R2, ZH2, d, H, H, rr, rr, zh, zh, zh, zh);
  const uint32_t I = small(HH, 4);
  uint32_t Jv, V;
  mul4(c, Jv, V, d, d1, H, I, a.x, I, H, I, H, I);
  const uint32_t X3 = sub<2>(c, R2, add(Jv, small(V, 2)));  // < 5.0004
  const uint32_t w = sub<3>(c, V, X3);
  uint32_t rw, yj;
  mul4(c, rw, yj, d, d1, rr, w, a.y, Jv, rr, w, rr, w);
  o.x = X3;
  o.y = sub<2>(c, rw, small(yj, 2));
  o.z = sub<2>(c, ZH2, add(zz, HH));
}

// x^(p-2) = (x^((p-3)/4))^4 x: the inverse of a nonzero x (every row, redundantly)
__device__ __forceinline__ uint32_t inv(const Ctx &c, uint32_t x) {
  uint32_t a = dfp::pow_pm3d4(x, c.t);
  a = dfp::mul(a, a, c.t);
  a = dfp::mul(a, a, c.t);
  return dfp::mul(a, x, c.t);
}
// Jacobian -> affine; infinity -> all-zero (blst's encoding).  Writes canonical engine words.
__device__ __forceinline__ void store_affine(const Ctx &c, g2a *out, const J &p) {
  if (is_inf(c, p)) {
    const uint32_t j = c.t.j;
    if (c.r == 0 && j < 12) {
      out->x.c0.l[j] = 0;
      out->x.c1.l[j] = 0;
      out->y.c0.l[j] = 0;
      out->y.c1.l[j] = 0;
    }
    return;
  }
  // 1/Z = conj(Z) / N(Z)
  uint32_t n, d0, d1, d2;
  const uint32_t X[4] = {p.z.c0, p.z.c0, p.z.c0, p.z.c0}, Z[4] = {p.z.c1, p.z.c1, p.z.c1, p.z.c1};
  mul4d(c, n, d0, d1, d2, X, X, Z, Z);
  const uint32_t ni = inv(c, n);
  f2 zi;
  mul4(c, zi.c0, zi.c1, d0, d1, p.z.c0, ni, sub<10>(c, 0u, p.z.c1), ni, p.z.c0, ni, p.z.c0, ni);
  uint32_t s0, sx;
  mul4(c, s0, sx, d0, d1, add(zi.c0, zi.c1), sub<2>(c, zi.c0, zi.c1), zi.c0, zi.c1, zi.c0, zi.c1,
       zi.c0, zi.c1);
  const f2 zi2 = sqr_of(s0, sx);
  // x = X zi2 and zi3 = zi2 zi as two dual-product pairs per coefficient
  f2 x, zi3;
  const f2 nzi2 = neg<2, 3>(c, zi2);
  {
    const uint32_t A[4] = {p.x.c0, p.x.c0, zi2.c0, zi2.c0}, B[4] = {zi2.c0, zi2.c1, zi.c0, zi.c1};
    const uint32_t C[4] = {p.x.c1, p.x.c1, zi2.c1, zi2.c1}, D[4] = {nzi2.c1, zi2.c0, sub<2>(c, 0u, zi.c1), zi.c0};
    mul4d(c, x.c0, x.c1, zi3.c0, zi3.c1, A, B, C, D);
  }
  f2 y;
  {
    const f2 nzi3 = neg<1, 1>(c, zi3);
    const uint32_t A[4] = {p.y.c0, p.y.c0, p.y.c0, p.y.c0}, B[4] = {zi3.c0, zi3.c1, zi3.c0, zi3.c1};
    const uint32_t C[4] = {p.y.c1, p.y.c1, p.y.c1, p.y.c1}, D[4] = {nzi3.c1, zi3.c0, nzi3.c1, zi3.c0};
    mul4d(c, y.c0, y.c1, d0, d1, A, B, C, D);
  }
  store4(c, x.c0, x.c1, y.c0, y.c1, out->x.c0.l, out->x.c1.l, out->y.c0.l, out->y.c1.l);
}

}  // namespace w4
}  // namespace gbls
