// Optimal-ate pairing pieces: Miller loop with projective line functions on the
// twist, and the final exponentiation (p^12-1)/r (easy part + Hayashida-Hayasaka-
// Teruya hard-part chain, which computes the 3rd power of the textbook map; the
// verdict "== 1" is unchanged because gcd(3, r) = 1).
//
// Replaces blst miller_loop_n / final_exp / PAIRING_FinalVerify reached from
// Signature::verify, fast_aggregate_verify and multi_verify
// (bls/src/signature.rs:47-60, 77-93, 95-129).
//
// No inversions on the Miller inputs: P comes straight from the Jacobian r*pk and is
// stored pre-scaled as (XZ, Y, Z^3), so line(P) ~ L0 Z^3 + L2 XZ + L3 Y (a factor
// Z^3 in Fp, killed by the final exponentiation); Q is homogeneous projective.
#pragma once
#include "bls_curve.h"

namespace gbls {

struct g1p {  // Miller-loop form of a G1 point (Jacobian (X,Y,Z) -> XZ, Y, Z^3)
  fp xz, y, z3;
};
struct g2h {  // homogeneous projective G2 point (x = X/Z, y = Y/Z)
  fp2 x, y, z;
};

HD void g1p_from_jac(g1p &r, const g1j &p) {
  if (jac_is_inf(p)) {
    fp_zero(r.xz);
    fp_zero(r.y);
    fp_zero(r.z3);
    return;
  }
  fp z2;
  fp_mul(r.xz, p.x, p.z);
  r.y = p.y;
  fp_sqr(z2, p.z);
  fp_mul(r.z3, z2, p.z);
}
HD void g1p_from_aff(g1p &r, const g1a &a) {
  if (aff_is_inf(a)) {
    fp_zero(r.xz);
    fp_zero(r.y);
    fp_zero(r.z3);
    return;
  }
  r.xz = a.x;
  r.y = a.y;
  fp_one(r.z3);
}
// Jacobian (X, Y, Z) -> homogeneous (X Z, Y, Z^3)
HD void g2h_from_jac(g2h &r, const g2j &p) {
  if (jac_is_inf(p)) {
    fp2_zero(r.x);
    fp2_one(r.y);
    fp2_zero(r.z);
    return;
  }
  fp2 z2;
  fp2_mul(r.x, p.x, p.z);
  r.y = p.y;
  fp2_sqr(z2, p.z);
  fp2_mul(r.z, z2, p.z);
}

// Doubling step on T (homogeneous projective on the twist), returning the line
// coefficients scaled so that line(P) = L0 + (L2 * xP) w^2 + (L3 * yP) w^3:
//   L0 = 3b'Z^2 - Y^2,  L2 = 3X^2,  L3 = -2YZ      (Miller loop)
HD void line_dbl(g2h &T, fp2 &L0, fp2 &L2, fp2 &L3) {
  const fp inv2 = fp_const(k::INV2_M);
  fp2 A, B, C, E, F, G, H, t;
  fp2_mul(A, T.x, T.y);
  fp2_mul_fp(A, A, inv2);  // XY/2
  fp2_sqr(B, T.y);         // Y^2
  fp2_sqr(C, T.z);         // Z^2
  fp2_mul3(E, C);
  fp2_mul(E, E, fp2_const(k::B2_C0, k::B2_C1));  // 3 b' Z^2
  fp2_mul3(F, E);
  fp2_add(t, T.y, T.z);
  fp2_sqr(H, t);
  fp2_sub(H, H, B);
  fp2_sub(H, H, C);  // 2YZ
  fp2_sub(L0, E, B);
  fp2_sqr(t, T.x);
  fp2_mul3(L2, t);
  fp2_neg(L3, H);
  fp2_sub(t, B, F);
  fp2_mul(T.x, A, t);
  fp2_add(G, B, F);
  fp2_mul_fp(G, G, inv2);
  fp2_sqr(G, G);
  fp2_sqr(t, E);
  fp2_mul3(t, t);
  fp2_sub(T.y, G, t);
  fp2_mul(T.z, B, H);
}

// Addition step T + Q, both homogeneous:  theta = Y1 Z2 - Y2 Z1, lambda = X1 Z2 - X2 Z1,
//   L0 = theta X2 - lambda Y2,  L2 = -theta Z2,  L3 = lambda Z2
// and T <- T + Q  (add-1998-cmo-2 with u = -theta, v = -lambda)
HD void line_add(g2h &T, const g2h &Q, fp2 &L0, fp2 &L2, fp2 &L3) {
  fp2 x1z2, y1z2, t, th, la;
  fp2_mul(x1z2, T.x, Q.z);
  fp2_mul(y1z2, T.y, Q.z);
  fp2_mul(t, Q.y, T.z);
  fp2_sub(th, y1z2, t);
  fp2_mul(t, Q.x, T.z);
  fp2_sub(la, x1z2, t);
  fp2_mul(L0, th, Q.x);
  fp2_mul(t, la, Q.y);
  fp2_sub(L0, L0, t);
  fp2_mul(L2, th, Q.z);
  fp2_neg(L2, L2);
  fp2_mul(L3, la, Q.z);
  // homogeneous addition
  fp2 uu, vv, vvv, R, z1z2, A;
  fp2_sqr(uu, th);  // u^2 = theta^2
  fp2_sqr(vv, la);  // v^2 = lambda^2
  fp2_mul(vvv, vv, la);
  fp2_neg(vvv, vvv);  // v^3 = -lambda^3
  fp2_mul(R, vv, x1z2);
  fp2_mul(z1z2, T.z, Q.z);
  fp2_mul(A, uu, z1z2);
  fp2_sub(A, A, vvv);
  fp2_sub(A, A, R);
  fp2_sub(A, A, R);
  fp2_mul(T.x, la, A);
  fp2_neg(T.x, T.x);  // X3 = v A
  fp2_sub(t, R, A);
  fp2_mul(t, th, t);
  fp2_neg(t, t);  // u (R - A)
  fp2_mul(R, vvv, y1z2);
  fp2_sub(T.y, t, R);
  fp2_mul(T.z, vvv, z1z2);
}

HD void apply_line(fp12 &f, const fp2 &L0, const fp2 &L2, const fp2 &L3, const g1p &P) {
  fp2 l0, l2, l3;
  fp2_mul_fp(l0, L0, P.z3);
  fp2_mul_fp(l2, L2, P.xz);
  fp2_mul_fp(l3, L3, P.y);
  fp12_mul_line(f, f, l0, l2, l3);
}

// f_{|x|,Q}(P), conjugated (x < 0).  Infinity on either side gives 1.
HD void miller_loop(fp12 &f, const g1p &P, const g2h &Q) {
  fp12_one(f);
  if (fp_is_zero(P.z3) || fp2_is_zero(Q.z)) return;
  g2h T = Q;
  fp2 L0, L2, L3;
  line_dbl(T, L0, L2, L3);  // first step: f = 1 -> no squaring
  {
    fp2 l0, l2, l3;
    fp2_mul_fp(l0, L0, P.z3);
    fp2_mul_fp(l2, L2, P.xz);
    fp2_mul_fp(l3, L3, P.y);
    fp2_zero(f.c0.c2);
    f.c0.c0 = l0;
    f.c0.c1 = l2;
    fp2_zero(f.c1.c0);
    f.c1.c1 = l3;
    fp2_zero(f.c1.c2);
  }
  for (int i = 61; i >= 0; i--) {
    if ((k::X_ABS >> (i + 1)) & 1) {  // addition belonging to the previous bit
      line_add(T, Q, L0, L2, L3);
      apply_line(f, L0, L2, L3, P);
    }
    line_dbl(T, L0, L2, L3);
    fp12_sqr(f, f);
    apply_line(f, L0, L2, L3, P);
  }
  fp12_conj(f, f);
}

// a^|x| then conjugate: a^x for a in the cyclotomic subgroup
HD void fp12_cyc_exp_x(fp12 &r, const fp12 &a) {
  fp12 acc = a;
  for (int i = 62; i >= 0; i--) {
    fp12_sqr(acc, acc);
    if ((k::X_ABS >> i) & 1) fp12_mul(acc, acc, a);
  }
  fp12_conj(r, acc);
}

// Final exponentiation, split in stages so each device kernel stays small:
//   easy:  F = f^((p^6-1)(p^2+1))
//   s1:    A = F^(x-1)            s2: A = A^(x-1)
//   s3:    B = A^(x+p)            s4: T = B^x
//   s5:    C = T^x frob2(B) conj(B)
//   s6:    R = C F^3   ( = f^(3 (p^12-1)/r) )
HD void fe_easy(fp12 &F, const fp12 &f) {
  fp12 t0, t1;
  fp12_inv(t0, f);
  fp12_conj(t1, f);
  fp12_mul(t1, t1, t0);
  fp12_frob2(t0, t1);
  fp12_mul(F, t0, t1);
}
HD void fe_s_xm1(fp12 &A, const fp12 &a) {  // a^(x-1)
  fp12 t0, t1;
  fp12_cyc_exp_x(t0, a);
  fp12_conj(t1, a);
  fp12_mul(A, t0, t1);
}
HD void fe_s_xpp(fp12 &B, const fp12 &a) {  // a^(x+p)
  fp12 t0, t1;
  fp12_cyc_exp_x(t0, a);
  fp12_frob(t1, a);
  fp12_mul(B, t0, t1);
}
HD void fe_s5(fp12 &C, const fp12 &T, const fp12 &B) {
  fp12 t0, t1;
  fp12_cyc_exp_x(t0, T);
  fp12_frob2(t1, B);
  fp12_mul(t0, t0, t1);
  fp12_conj(t1, B);
  fp12_mul(C, t0, t1);
}
HD void fe_s6(fp12 &R, const fp12 &C, const fp12 &F) {
  fp12 t0;
  fp12_sqr(t0, F);
  fp12_mul(t0, t0, F);
  fp12_mul(R, C, t0);
}
// whole chain (host harness / reference composition of the stages)
HD void final_exp(fp12 &r, const fp12 &f) {
  fp12 F, A, B, T, C;
  fe_easy(F, f);
  fe_s_xm1(A, F);
  fe_s_xm1(A, A);
  fe_s_xpp(B, A);
  fp12_cyc_exp_x(T, B);
  fe_s5(C, T, B);
  fe_s6(r, C, F);
}

}  // namespace gbls
