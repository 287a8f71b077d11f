// Quad gangs: four adjacent lanes (one DPP quad) cooperate on one G2 point.
//
// A lane-per-point G2 doubling is a serial chain of 2 Fp2 products and 5 Fp2 squarings
// (16 Fp products).  Its dependency DAG is only three levels deep, so a quad runs each
// level's independent Fp2 operations side by side, one per lane, as ONE instruction
// stream with per-lane operands (v_cndmask selects), and shares the results with DPP
// quad_perm broadcasts (a VALU move, no LDS):
//
//   level 1: X^2, Y^2, (Y+Z)^2, Z^2     -> A, B, 2YZ = (Y+Z)^2 - B - Z^2
//   level 2: B^2, (X+B)^2, E^2 (E = 3A) -> C, D = 2((X+B)^2 - A - C), F
//   level 3: E (D - X3)                 (Karatsuba terms on lanes 0-2)
//
// Critical path 2 + 2 + 1 = 5 Fp products instead of 16 (the level-3 product's three
// Karatsuba terms go to three lanes, gang_fp2_mul).  Every lane of the quad ends
// holding the same point, so the rest of the code (additions, psi, to-affine) runs
// unchanged and redundantly.  Used by cofactor clearing, the dominant stage of
// hash_to_G2 (a13; blst Hash_to_G2 -> clear_cofactor via Budroni-Pintore).
#pragma once
#include "bls_curve.h"

namespace gbls {

template <int K>
__device__ __forceinline__ uint32_t quad_bcast(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, K * 0x55, 0xf, 0xf, false);
}
template <int K>
__device__ __forceinline__ void fp2_quad_bcast(fp2 &r, const fp2 &a) {
#pragma unroll
  for (int i = 0; i < 12; i++) {
    r.c0.l[i] = quad_bcast<K>(a.c0.l[i]);
    r.c1.l[i] = quad_bcast<K>(a.c1.l[i]);
  }
}
template <int K>
__device__ __forceinline__ void fp_quad_bcast(fp &r, const fp &a) {
#pragma unroll
  for (int i = 0; i < 12; i++) r.l[i] = quad_bcast<K>(a.l[i]);
}
// Fp2 product with its three Karatsuba Fp products spread over lanes 0-2 of the quad
// (lane 3 duplicates lane 2): one Fp product of latency instead of three.  r = a b in
// every lane; r may alias a or b.
__device__ __forceinline__ void gang_fp2_mul(fp2 &r, const fp2 &a, const fp2 &b, int q) {
  fp x, y, p, t0, t1, t2;
  fp sa, sb;
  fp_add_lazy(sa, a.c0, a.c1);  // < 2p: a Montgomery operand
  fp_add_lazy(sb, b.c0, b.c1);
#pragma unroll
  for (int i = 0; i < 12; i++) {
    x.l[i] = q == 0 ? a.c0.l[i] : (q == 1 ? a.c1.l[i] : sa.l[i]);
    y.l[i] = q == 0 ? b.c0.l[i] : (q == 1 ? b.c1.l[i] : sb.l[i]);
  }
  fp_mul(p, x, y);
  fp_quad_bcast<0>(t0, p);
  fp_quad_bcast<1>(t1, p);
  fp_quad_bcast<2>(t2, p);
  fp_sub(r.c0, t0, t1);
  fp_add(t0, t0, t1);
  fp_sub(r.c1, t2, t0);
}
// r = q==0 ? a : q==1 ? b : q==2 ? c : d, limb-wise (no branches)
__device__ __forceinline__ void fp2_sel4(fp2 &r, int q, const fp2 &a, const fp2 &b, const fp2 &c,
                                         const fp2 &d) {
#pragma unroll
  for (int i = 0; i < 12; i++) {
    uint32_t x0 = q == 0 ? a.c0.l[i] : b.c0.l[i];
    uint32_t y0 = q == 2 ? c.c0.l[i] : d.c0.l[i];
    r.c0.l[i] = q < 2 ? x0 : y0;
    uint32_t x1 = q == 0 ? a.c1.l[i] : b.c1.l[i];
    uint32_t y1 = q == 2 ? c.c1.l[i] : d.c1.l[i];
    r.c1.l[i] = q < 2 ? x1 : y1;
  }
}

// dbl-2009-l (a = 0) across a quad; q = lane & 3.  r may alias p.
__device__ __forceinline__ void gang_dbl(g2j &r, const g2j &p, int q) {
  fp2 in, s, A, B, W, Z2, E, t;
  f_add(t, p.y, p.z);
  fp2_sel4(in, q, p.x, p.y, t, p.z);
  fp2_sqr(s, in);
  fp2_quad_bcast<0>(A, s);
  fp2_quad_bcast<1>(B, s);
  fp2_quad_bcast<2>(W, s);
  fp2_quad_bcast<3>(Z2, s);
  f_add(t, p.x, B);  // X + B          (p.x dead)
  f_sub(W, W, B);
  f_sub(r.z, W, Z2);  // Z3 = (Y+Z)^2 - Y^2 - Z^2 = 2YZ
  f_dbl(E, A);
  f_add(E, E, A);  // E = 3A
  fp2_sel4(in, q, B, t, E, E);
  fp2_sqr(s, in);
  fp2 C, U, F;
  fp2_quad_bcast<0>(C, s);
  fp2_quad_bcast<1>(U, s);
  fp2_quad_bcast<2>(F, s);
  f_sub(U, U, A);
  f_sub(U, U, C);
  f_dbl(U, U);        // D
  f_sub(F, F, U);
  f_sub(r.x, F, U);   // X3 = F - 2D
  f_sub(t, U, r.x);
  gang_fp2_mul(t, E, t, q);  // E (D - X3)
  f_dbl(C, C);
  f_dbl(C, C);
  f_dbl(C, C);
  f_sub(r.y, t, C);   // Y3 = E (D - X3) - 8C
}

// add-2007-bl (jac_add, bls_curve.h) across a quad, r = a + b, r may alias a.  Serial:
// 11 Fp2 products + 5 squarings; here five levels of one Fp2 product each:
//   level 1: Z1^2, Z2^2, Y1 Z2, Y2 Z1
//   level 2: U1 = X1 Z2Z2, U2 = X2 Z1Z1, S1 = Y1Z2 Z2Z2, S2 = Y2Z1 Z1Z1   (H, r)
//   level 3: I = (2H)^2, r^2, (Z1 + Z2)^2
//   level 4: J = H I, V = U1 I, Z3 = 2 Z1 Z2 H
//   level 5: r (V - X3), S1 J
// The degenerate branches depend only on values every lane of the quad shares.
__device__ __forceinline__ void gang_add(g2j &r, const g2j &a, const g2j &b, int q) {
  if (jac_is_inf(b)) {
    r = a;
    return;
  }
  if (jac_is_inf(a)) {
    r = b;
    return;
  }
  fp2 x, y, s, Z1Z1, Z2Z2, U1, U2, S1, S2;
  fp2_sel4(x, q, a.z, b.z, a.y, b.y);
  fp2_sel4(y, q, a.z, b.z, b.z, a.z);
  fp2_mul(s, x, y);
  fp2_quad_bcast<0>(Z1Z1, s);
  fp2_quad_bcast<1>(Z2Z2, s);
  fp2_quad_bcast<2>(S1, s);
  fp2_quad_bcast<3>(S2, s);
  fp2_sel4(x, q, a.x, b.x, S1, S2);
  fp2_sel4(y, q, Z2Z2, Z1Z1, Z2Z2, Z1Z1);
  fp2_mul(s, x, y);
  fp2_quad_bcast<0>(U1, s);
  fp2_quad_bcast<1>(U2, s);
  fp2_quad_bcast<2>(S1, s);
  fp2_quad_bcast<3>(S2, s);
  fp2 H, R, t;
  fp2_sub(H, U2, U1);
  fp2_sub(R, S2, S1);
  fp2_add(R, R, R);  // r = 2 (S2 - S1)
  if (fp2_is_zero(H)) {
    if (fp2_is_zero(R)) {
      gang_dbl(r, b, q);
    } else {
      jac_set_inf(r);
    }
    return;
  }
  fp2 H2, ZZ, I, R2, Zs;
  fp2_add(H2, H, H);
  fp2_add(ZZ, a.z, b.z);
  fp2_sel4(x, q, H2, R, ZZ, ZZ);
  fp2_mul(s, x, x);
  fp2_quad_bcast<0>(I, s);
  fp2_quad_bcast<1>(R2, s);
  fp2_quad_bcast<2>(Zs, s);
  fp2_sub(Zs, Zs, Z1Z1);
  fp2_sub(Zs, Zs, Z2Z2);  // 2 Z1 Z2
  fp2 J, V;
  fp2_sel4(x, q, H, U1, Zs, Zs);
  fp2_sel4(y, q, I, I, H, H);
  fp2_mul(s, x, y);
  fp2_quad_bcast<0>(J, s);
  fp2_quad_bcast<1>(V, s);
  fp2_quad_bcast<2>(r.z, s);  // Z3 = 2 Z1 Z2 H   (a.z, b.z dead)
  fp2_sub(t, R2, J);
  fp2_sub(t, t, V);
  fp2_sub(r.x, t, V);         // X3 = r^2 - J - 2V
  fp2_sub(t, V, r.x);
  fp2_sel4(x, q, R, S1, R, S1);
  fp2_sel4(y, q, t, J, t, J);
  fp2_mul(s, x, y);
  fp2_quad_bcast<0>(t, s);
  fp2_quad_bcast<1>(S1, s);
  fp2_add(S1, S1, S1);
  fp2_sub(r.y, t, S1);        // Y3 = r (V - X3) - 2 S1 J
}

// ---------------------------------------------------------------- G1 (Fp) quad gangs
__device__ __forceinline__ void fp_sel4(fp &r, int q, const fp &a, const fp &b, const fp &c,
                                        const fp &d) {
#pragma unroll
  for (int i = 0; i < 12; i++) {
    uint32_t x = q == 0 ? a.l[i] : b.l[i];
    uint32_t y = q == 2 ? c.l[i] : d.l[i];
    r.l[i] = q < 2 ? x : y;
  }
}
// dbl-2009-l over Fp across a quad: levels X^2 Y^2 (Y+Z)^2 Z^2 | B^2 (X+B)^2 E^2 | E (D-X3)
// (3 Fp products deep instead of 7).  r may alias p.
__device__ __forceinline__ void gang1_dbl(g1j &r, const g1j &p, int q) {
  fp in, s, A, B, W, Z2, E, t;
  fp_add(t, p.y, p.z);
  fp_sel4(in, q, p.x, p.y, t, p.z);
  fp_sqr(s, in);
  fp_quad_bcast<0>(A, s);
  fp_quad_bcast<1>(B, s);
  fp_quad_bcast<2>(W, s);
  fp_quad_bcast<3>(Z2, s);
  fp_add(t, p.x, B);
  fp_sub(W, W, B);
  fp_sub(r.z, W, Z2);  // Z3 = 2YZ
  fp_add(E, A, A);
  fp_add(E, E, A);     // E = 3A
  fp_sel4(in, q, B, t, E, E);
  fp_sqr(s, in);
  fp C, U, F;
  fp_quad_bcast<0>(C, s);
  fp_quad_bcast<1>(U, s);
  fp_quad_bcast<2>(F, s);
  fp_sub(U, U, A);
  fp_sub(U, U, C);
  fp_add(U, U, U);     // D
  fp_sub(F, F, U);
  fp_sub(r.x, F, U);   // X3 = F - 2D
  fp_sub(t, U, r.x);
  fp_mul(t, E, t);     // E (D - X3), the same in every lane
  fp_add(C, C, C);
  fp_add(C, C, C);
  fp_add(C, C, C);
  fp_sub(r.y, t, C);   // Y3 = E (D - X3) - 8C
}
// add-2007-bl over Fp across a quad (5 Fp products deep instead of 16), r = a + b,
// r may alias a.  The degenerate branches depend only on values the quad shares.
__device__ __forceinline__ void gang1_add(g1j &r, const g1j &a, const g1j &b, int q) {
  if (jac_is_inf(b)) {
    r = a;
    return;
  }
  if (jac_is_inf(a)) {
    r = b;
    return;
  }
  fp x, y, s, Z1Z1, Z2Z2, U1, U2, S1, S2;
  fp_sel4(x, q, a.z, b.z, a.y, b.y);
  fp_sel4(y, q, a.z, b.z, b.z, a.z);
  fp_mul(s, x, y);
  fp_quad_bcast<0>(Z1Z1, s);
  fp_quad_bcast<1>(Z2Z2, s);
  fp_quad_bcast<2>(S1, s);
  fp_quad_bcast<3>(S2, s);
  fp_sel4(x, q, a.x, b.x, S1, S2);
  fp_sel4(y, q, Z2Z2, Z1Z1, Z2Z2, Z1Z1);
  fp_mul(s, x, y);
  fp_quad_bcast<0>(U1, s);
  fp_quad_bcast<1>(U2, s);
  fp_quad_bcast<2>(S1, s);
  fp_quad_bcast<3>(S2, s);
  fp H, R, t;
  fp_sub(H, U2, U1);
  fp_sub(R, S2, S1);
  fp_add(R, R, R);
  if (fp_is_zero(H)) {
    if (fp_is_zero(R)) {
      gang1_dbl(r, b, q);
    } else {
      jac_set_inf(r);
    }
    return;
  }
  fp H2, ZZ, I, R2, Zs;
  fp_add(H2, H, H);
  fp_add(ZZ, a.z, b.z);
  fp_sel4(x, q, H2, R, ZZ, ZZ);
  fp_sqr(s, x);
  fp_quad_bcast<0>(I, s);
  fp_quad_bcast<1>(R2, s);
  fp_quad_bcast<2>(Zs, s);
  fp_sub(Zs, Zs, Z1Z1);
  fp_sub(Zs, Zs, Z2Z2);  // 2 Z1 Z2
  fp J, V;
  fp_sel4(x, q, H, U1, Zs, Zs);
  fp_sel4(y, q, I, I, H, H);
  fp_mul(s, x, y);
  fp_quad_bcast<0>(J, s);
  fp_quad_bcast<1>(V, s);
  fp_quad_bcast<2>(r.z, s);  // Z3 = 2 Z1 Z2 H
  fp_sub(t, R2, J);
  fp_sub(t, t, V);
  fp_sub(r.x, t, V);         // X3 = R^2 - J - 2V
  fp_sub(t, V, r.x);
  fp_sel4(x, q, R, S1, R, S1);
  fp_sel4(y, q, t, J, t, J);
  fp_mul(s, x, y);
  fp_quad_bcast<0>(t, s);
  fp_quad_bcast<1>(S1, s);
  fp_add(S1, S1, S1);
  fp_sub(r.y, t, S1);        // Y3 = R (V - X3) - 2 S1 J
}

// ---------------------------------------------------------------- 16-lane row gangs
// For small launches (a lone 4096-set batch fills 256 of 1024 SIMDs with quads): one DPP
// row (16 lanes) per point.  Each dependency level issues up to
// four Fp2 products at once, quad j of the row computing product j as three Karatsuba Fp
// products (lanes k = 0, 1, 2; lane 3 repeats 2), so a level costs ONE Fp product of
// latency: Miller doubling step 3 levels (quad: 7 products), addition step 4 (quad: 12).
// Products are recombined inside the quad (quad_perm), then shared with the row by
// row_newbcast: VALU moves, no LDS.  Every lane ends holding the same values.  (Row
// doublings / additions for cofactor clearing measured slower than the quad ones: 2.01 vs
// 1.91 ms at 4096 sets, the selects and broadcasts outweighing 3 vs 5 product levels.)
template <int L>
__device__ __forceinline__ uint32_t row_bcast(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x150 + L, 0xf, 0xf, false);
}
template <int L>
__device__ __forceinline__ void fp2_row_bcast(fp2 &r, const fp2 &a) {
#pragma unroll
  for (int i = 0; i < 12; i++) {
    r.c0.l[i] = row_bcast<L>(a.c0.l[i]);
    r.c1.l[i] = row_bcast<L>(a.c1.l[i]);
  }
}
// R_j = A_j B_j (j < 4) in every lane of the row; l = lane & 15.  R may alias inputs.
__device__ __forceinline__ void row_mul4(fp2 &R0, fp2 &R1, fp2 &R2, fp2 &R3, const fp2 &A0,
                                         const fp2 &A1, const fp2 &A2, const fp2 &A3,
                                         const fp2 &B0, const fp2 &B1, const fp2 &B2,
                                         const fp2 &B3, int l) {
  const int j = l >> 2, k = l & 3;
  fp2 a, b;
  fp2_sel4(a, j, A0, A1, A2, A3);
  fp2_sel4(b, j, B0, B1, B2, B3);
  fp x, y, sa, sb;
  fp_add_lazy(sa, a.c0, a.c1);  // < 2p: a Montgomery operand
  fp_add_lazy(sb, b.c0, b.c1);
#pragma unroll
  for (int i = 0; i < 12; i++) {
    x.l[i] = k == 0 ? a.c0.l[i] : (k == 1 ? a.c1.l[i] : sa.l[i]);
    y.l[i] = k == 0 ? b.c0.l[i] : (k == 1 ? b.c1.l[i] : sb.l[i]);
  }
  fp p, t0, t1, t2;
  fp_mul(p, x, y);
  fp_quad_bcast<0>(t0, p);
  fp_quad_bcast<1>(t1, p);
  fp_quad_bcast<2>(t2, p);
  fp2 c;
  fp_sub(c.c0, t0, t1);
  fp_add(t0, t0, t1);
  fp_sub(c.c1, t2, t0);
  fp2_row_bcast<0>(R0, c);
  fp2_row_bcast<4>(R1, c);
  fp2_row_bcast<8>(R2, c);
  fp2_row_bcast<12>(R3, c);
}

// dbl-2009-l across a row (gang_dbl's three levels), r may alias p
__device__ __forceinline__ void row_dbl(g2j &r, const g2j &p, int l) {
  fp2 t, A, B, W, Z2;
  f_add(t, p.y, p.z);
  row_mul4(A, B, W, Z2, p.x, p.y, t, p.z, p.x, p.y, t, p.z, l);
  fp2 E, C, U, F, x;
  f_add(t, p.x, B);  // X + B
  f_sub(W, W, B);
  f_sub(r.z, W, Z2);  // Z3 = 2YZ
  f_dbl(E, A);
  f_add(E, E, A);     // E = 3A
  row_mul4(C, U, F, x, B, t, E, E, B, t, E, E, l);
  f_sub(U, U, A);
  f_sub(U, U, C);
  f_dbl(U, U);        // D
  f_sub(F, F, U);
  f_sub(r.x, F, U);   // X3 = F - 2D
  f_sub(t, U, r.x);
  row_mul4(t, x, x, x, E, E, E, E, t, t, t, t, l);  // E (D - X3)
  f_dbl(C, C);
  f_dbl(C, C);
  f_dbl(C, C);
  f_sub(r.y, t, C);   // Y3 = E (D - X3) - 8C
}

// add-2007-bl across a row (gang_add's five levels), r = a + b, r may alias a
__device__ __forceinline__ void row_add(g2j &r, const g2j &a, const g2j &b, int l) {
  if (jac_is_inf(b)) {
    r = a;
    return;
  }
  if (jac_is_inf(a)) {
    r = b;
    return;
  }
  fp2 Z1Z1, Z2Z2, U1, U2, S1, S2;
  row_mul4(Z1Z1, Z2Z2, S1, S2, a.z, b.z, a.y, b.y, a.z, b.z, b.z, a.z, l);
  row_mul4(U1, U2, S1, S2, a.x, b.x, S1, S2, Z2Z2, Z1Z1, Z2Z2, Z1Z1, l);
  fp2 H, R, t, w;
  fp2_sub(H, U2, U1);
  fp2_sub(R, S2, S1);
  fp2_add(R, R, R);  // r = 2 (S2 - S1)
  if (fp2_is_zero(H)) {
    if (fp2_is_zero(R)) {
      row_dbl(r, b, l);
    } else {
      jac_set_inf(r);
    }
    return;
  }
  fp2 H2, ZZ, I, R2, Zs;
  fp2_add(H2, H, H);
  fp2_add(ZZ, a.z, b.z);
  row_mul4(I, R2, Zs, w, H2, R, ZZ, ZZ, H2, R, ZZ, ZZ, l);
  fp2_sub(Zs, Zs, Z1Z1);
  fp2_sub(Zs, Zs, Z2Z2);  // 2 Z1 Z2
  fp2 J, V;
  row_mul4(J, V, r.z, w, H, U1, Zs, Zs, I, I, H, H, l);  // Z3 = 2 Z1 Z2 H
  fp2_sub(t, R2, J);
  fp2_sub(t, t, V);
  fp2_sub(r.x, t, V);  // X3 = r^2 - J - 2V
  fp2_sub(t, V, r.x);
  row_mul4(t, S1, w, w, R, S1, R, S1, t, J, t, J, l);
  fp2_add(S1, S1, S1);
  fp2_sub(r.y, t, S1);  // Y3 = r (V - X3) - 2 S1 J
}

// [|x|]P with row doublings and additions
__device__ __forceinline__ void row_mul_by_xabs(g2j &r, const g2j &p, int l) {
  g2j acc = p;
  for (int i = 62; i >= 0; i--) {
    row_dbl(acc, acc, l);
    if ((k::X_ABS >> i) & 1) row_add(acc, acc, p, l);
  }
  r = acc;
}

// [|x|]P with quad-cooperative doublings and additions
__device__ __forceinline__ void gang_mul_by_xabs(g2j &r, const g2j &p, int q) {
  g2j acc = p;
  for (int i = 62; i >= 0; i--) {
    gang_dbl(acc, acc, q);
    if ((k::X_ABS >> i) & 1) gang_add(acc, acc, p, q);
  }
  r = acc;
}

}  // namespace gbls

#ifdef GBLS_GANG_LINES
namespace gbls {

// Miller-loop doubling step (line_dbl, bls_pairing.h) across a quad.  Serial: 3 Fp2
// products + 5 squarings; here three levels of one Fp2 product each:
//   level 1: X Y, Y^2, Z^2, X^2
//   level 2: A (B - F), G^2, E^2, Y Z      (A = XY/2, E = 3b'Z^2, F = 3E, G = (B+F)/2)
//   level 3: Z3 = B H                      (H = 2YZ, Karatsuba terms on lanes 0-2)
// Line coefficients L0 = E - B, L2 = 3X^2, L3 = -H, as line_dbl.
__device__ __forceinline__ void gang_line_dbl(g2h &T, fp2 &L0, fp2 &L2, fp2 &L3, int q) {
  fp2 a, b, s, A, B, C, X2;
  fp2_sel4(a, q, T.x, T.y, T.z, T.x);
  fp2_sel4(b, q, T.y, T.y, T.z, T.x);
  fp2_mul(s, a, b);
  fp2_quad_bcast<0>(A, s);
  fp2_quad_bcast<1>(B, s);
  fp2_quad_bcast<2>(C, s);
  fp2_quad_bcast<3>(X2, s);
  fp2_half(A, A);     // XY/2
  fp2 E, F, G, t1;
  fp2_mul_3b(E, C);   // 3b'Z^2
  fp2_add(F, E, E);
  fp2_add(F, F, E);   // 3E
  fp2_sub(L0, E, B);
  fp2_mul3(L2, X2);
  fp2_sub(t1, B, F);
  fp2_add(G, B, F);
  fp2_half(G, G);
  fp2_sel4(a, q, A, G, E, T.y);
  fp2_sel4(b, q, t1, G, E, T.z);
  fp2_mul(s, a, b);
  fp2 X3, G2, E2, H;
  fp2_quad_bcast<0>(X3, s);
  fp2_quad_bcast<1>(G2, s);
  fp2_quad_bcast<2>(E2, s);
  fp2_quad_bcast<3>(H, s);
  fp2_add(H, H, H);   // 2YZ
  fp2_neg(L3, H);
  T.x = X3;           // X3 = A (B - F)
  fp2_mul3(E2, E2);
  fp2_sub(T.y, G2, E2);  // Y3 = G^2 - 3E^2
  gang_fp2_mul(T.z, B, H, q);  // Z3 = B H
}

// Miller-loop addition step (line_add_aff, bls_pairing.h) across a quad, four levels of
// one Fp2 product per lane (serial: 11 products + 2 squarings):
//   level 1: y2 Z1, x2 Z1                       -> theta, lambda
//   level 2: theta x2, lambda y2, theta^2, lambda^2
//   level 3: lambda^3, lambda^2 X1, theta^2 Z1   -> A
//   level 4: lambda A, theta (R - A), lambda^3 Y1, lambda^3 Z1
__device__ __forceinline__ void gang_line_add_aff(g2h &T, const g2a &Q, fp2 &L0, fp2 &L2, fp2 &L3,
                                                  int q) {
  fp2 a, b, s, yZ, xZ, th, la;
  fp2_sel4(a, q, Q.y, Q.x, Q.y, Q.x);
  fp2_mul(s, a, T.z);
  fp2_quad_bcast<0>(yZ, s);
  fp2_quad_bcast<1>(xZ, s);
  fp2_sub(th, T.y, yZ);
  fp2_sub(la, T.x, xZ);
  fp2_sel4(a, q, th, la, th, la);
  fp2_sel4(b, q, Q.x, Q.y, th, la);
  fp2_mul(s, a, b);
  fp2 P0, P1, uu, vv;
  fp2_quad_bcast<0>(P0, s);
  fp2_quad_bcast<1>(P1, s);
  fp2_quad_bcast<2>(uu, s);
  fp2_quad_bcast<3>(vv, s);
  fp2_sub(L0, P0, P1);  // theta x2 - lambda y2
  fp2_neg(L2, th);
  L3 = la;
  fp2_sel4(a, q, vv, vv, uu, uu);
  fp2_sel4(b, q, la, T.x, T.z, T.z);
  fp2_mul(s, a, b);
  fp2 vvv, R, A, t;
  fp2_quad_bcast<0>(vvv, s);
  fp2_quad_bcast<1>(R, s);
  fp2_quad_bcast<2>(A, s);
  fp2_neg(vvv, vvv);    // v^3 = -lambda^3
  fp2_sub(A, A, vvv);
  fp2_sub(A, A, R);
  fp2_sub(A, A, R);
  fp2_sub(t, R, A);
  fp2_sel4(a, q, la, th, vvv, vvv);
  fp2_sel4(b, q, A, t, T.y, T.z);
  fp2_mul(s, a, b);
  fp2 X3, U, R2;
  fp2_quad_bcast<0>(X3, s);
  fp2_quad_bcast<1>(U, s);
  fp2_quad_bcast<2>(R2, s);
  fp2_quad_bcast<3>(T.z, s);  // Z3 = v^3 Z1
  fp2_neg(T.x, X3);           // X3 = v A
  fp2_neg(U, U);              // u (R - A)
  fp2_sub(T.y, U, R2);
}

// Miller doubling step across a row (gang_line_dbl's levels): X Y, Y^2, Z^2, X^2 |
// A (B - F), G^2, E^2, Y Z | B H
__device__ __forceinline__ void row_line_dbl(g2h &T, fp2 &L0, fp2 &L2, fp2 &L3, int l) {
  fp2 A, B, C, X2;
  row_mul4(A, B, C, X2, T.x, T.y, T.z, T.x, T.y, T.y, T.z, T.x, l);
  fp2_half(A, A);     // XY/2
  fp2 E, F, G, t1;
  fp2_mul_3b(E, C);   // 3b'Z^2
  fp2_add(F, E, E);
  fp2_add(F, F, E);   // 3E
  fp2_sub(L0, E, B);
  fp2_mul3(L2, X2);
  fp2_sub(t1, B, F);
  fp2_add(G, B, F);
  fp2_half(G, G);
  fp2 X3, G2, E2, H;
  row_mul4(X3, G2, E2, H, A, G, E, T.y, t1, G, E, T.z, l);
  fp2_add(H, H, H);   // 2YZ
  fp2_neg(L3, H);
  T.x = X3;           // X3 = A (B - F)
  fp2_mul3(E2, E2);
  fp2_sub(T.y, G2, E2);  // Y3 = G^2 - 3E^2
  fp2 w;
  row_mul4(T.z, w, w, w, B, B, B, B, H, H, H, H, l);  // Z3 = B H
}

// Miller addition step across a row (gang_line_add_aff's four levels)
__device__ __forceinline__ void row_line_add_aff(g2h &T, const g2a &Q, fp2 &L0, fp2 &L2, fp2 &L3,
                                                 int l) {
  fp2 yZ, xZ, th, la, w;
  row_mul4(yZ, xZ, w, w, Q.y, Q.x, Q.y, Q.x, T.z, T.z, T.z, T.z, l);
  fp2_sub(th, T.y, yZ);
  fp2_sub(la, T.x, xZ);
  fp2 P0, P1, uu, vv;
  row_mul4(P0, P1, uu, vv, th, la, th, la, Q.x, Q.y, th, la, l);
  fp2_sub(L0, P0, P1);  // theta x2 - lambda y2
  fp2_neg(L2, th);
  L3 = la;
  fp2 vvv, R, A, t;
  row_mul4(vvv, R, A, w, vv, vv, uu, uu, la, T.x, T.z, T.z, l);
  fp2_neg(vvv, vvv);    // v^3 = -lambda^3
  fp2_sub(A, A, vvv);
  fp2_sub(A, A, R);
  fp2_sub(A, A, R);
  fp2_sub(t, R, A);
  fp2 X3, U, R2;
  row_mul4(X3, U, R2, T.z, la, th, vvv, vvv, A, t, T.y, T.z, l);  // Z3 = v^3 Z1
  fp2_neg(T.x, X3);     // X3 = v A
  fp2_neg(U, U);        // u (R - A)
  fp2_sub(T.y, U, R2);
}

}  // namespace gbls
#endif
