// Optimal-ate pairing pieces: Miller loop with projective line functions on the
// twist, and the final exponentiation (p^12-1)/r (easy part + Hayashida-Hayasaka-
// Teruya hard-part chain, which computes the 3rd power of the textbook map; the
// verdict "== 1" is unchanged because gcd(3, r) = 1).
//
// Replaces blst miller_loop_n / final_exp / PAIRING_FinalVerify reached from
// Signature::verify, fast_aggregate_verify and multi_verify
// (bls/src/signature.rs:47-60, 77-93, 95-129).
#pragma once
#include "bls_curve.h"

namespace gbls {

// Doubling step on T (homogeneous projective on the twist), returning the line
// coefficients scaled so that line(P) = L0 + (L2 * xP) w^2 + (L3 * yP) w^3:
//   L0 = 3b'Z^2 - Y^2,  L2 = 3X^2,  L3 = -2YZ      (Miller loop)
HD void line_dbl(g2j &T, fp2 &L0, fp2 &L2, fp2 &L3) {
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
  // T = 2T
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

// Mixed addition step T + Q (Q affine): theta = Y - yQ Z, lambda = X - xQ Z,
//   L0 = theta xQ - lambda yQ,  L2 = -theta,  L3 = lambda
HD void line_add(g2j &T, const g2a &Q, fp2 &L0, fp2 &L2, fp2 &L3) {
  fp2 th, la, C, D, E, F, G, H, t;
  fp2_mul(t, Q.y, T.z);
  fp2_sub(th, T.y, t);
  fp2_mul(t, Q.x, T.z);
  fp2_sub(la, T.x, t);
  fp2_mul(L0, th, Q.x);
  fp2_mul(t, la, Q.y);
  fp2_sub(L0, L0, t);
  fp2_neg(L2, th);
  L3 = la;
  fp2_sqr(C, th);
  fp2_sqr(D, la);
  fp2_mul(E, la, D);
  fp2_mul(F, T.z, C);
  fp2_mul(G, T.x, D);
  fp2_add(H, E, F);
  fp2_sub(H, H, G);
  fp2_sub(H, H, G);
  fp2_mul(T.x, la, H);
  fp2_sub(t, G, H);
  fp2_mul(t, th, t);
  fp2_mul(C, E, T.y);
  fp2_sub(T.y, t, C);
  fp2_mul(T.z, T.z, E);
}

HD void apply_line(fp12 &f, const fp2 &L0, const fp2 &L2, const fp2 &L3, const g1a &P) {
  fp2 l2, l3;
  fp2_mul_fp(l2, L2, P.x);
  fp2_mul_fp(l3, L3, P.y);
  fp12_mul_line(f, f, L0, l2, l3);
}

HDNI void miller_add_step(fp12 &f, g2j &T, const g2a &Q, const g1a &P) {
  fp2 L0, L2, L3;
  line_add(T, Q, L0, L2, L3);
  apply_line(f, L0, L2, L3, P);
}

// f_{|x|,Q}(P), conjugated (x < 0).  Infinity on either side gives 1.
HDNI void miller_loop(fp12 &f, const g1a &P, const g2a &Q) {
  fp12_one(f);
  if (aff_is_inf(P) || aff_is_inf(Q)) return;
  g2j T;
  T.x = Q.x;
  T.y = Q.y;
  fp2_one(T.z);
  fp2 L0, L2, L3;
  bool first = true;
  for (int i = 62; i >= 0; i--) {
    line_dbl(T, L0, L2, L3);
    if (!first) fp12_sqr(f, f);
    first = false;
    apply_line(f, L0, L2, L3, P);
    if ((k::X_ABS >> i) & 1) miller_add_step(f, T, Q, P);
  }
  fp12_conj(f, f);
}

// a^|x| then conjugate: a^x for a in the cyclotomic subgroup
HDNI void fp12_cyc_exp_x(fp12 &r, const fp12 &a) {
  fp12 acc = a;
  for (int i = 62; i >= 0; i--) {
    fp12_sqr_n(acc, acc);
    if ((k::X_ABS >> i) & 1) fp12_mul_n(acc, acc, a);
  }
  fp12_conj(r, acc);
}

// f^(3 (p^12-1)/r)
HDNI void final_exp(fp12 &r, const fp12 &fin) {
  fp12 f, t0, t1;
  // easy part: f^(p^6-1)(p^2+1)
  fp12_inv_n(t0, fin);
  fp12_conj(f, fin);
  fp12_mul_n(f, f, t0);
  fp12_frob2_n(t0, f);
  fp12_mul_n(f, t0, f);
  // hard part: 3 Lambda = (x-1)^2 (x+p) (x^2+p^2-1) + 3
  fp12 a, b, c;
  fp12_cyc_exp_x(t0, f);
  fp12_conj(t1, f);
  fp12_mul_n(a, t0, t1);  // f^(x-1)
  fp12_cyc_exp_x(t0, a);
  fp12_conj(t1, a);
  fp12_mul_n(a, t0, t1);  // f^((x-1)^2)
  fp12_cyc_exp_x(t0, a);
  fp12_frob_n(t1, a);
  fp12_mul_n(b, t0, t1);  // a^(x+p)
  fp12_cyc_exp_x(t0, b);
  fp12_cyc_exp_x(t0, t0);
  fp12_frob2_n(t1, b);
  fp12_mul_n(c, t0, t1);
  fp12_conj(t1, b);
  fp12_mul_n(c, c, t1);  // b^(x^2+p^2-1)
  fp12_sqr_n(t0, f);
  fp12_mul_n(t0, t0, f);
  fp12_mul_n(r, c, t0);
}

}  // namespace gbls
