// Optimal-ate pairing pieces (BLS12-381, x = -0xd201000000010000).
//
// Replaces blst miller_loop_n / final_exp / PAIRING_FinalVerify reached from
// Signature::verify, fast_aggregate_verify and multi_verify (bls/src/signature.rs:47-60,
// 77-93, 95-129).  The device pipeline splits the Miller loop of a batch into
//   (1) per pair: the 68 line functions of T = Q along |x| ("events": 63 doublings,
//       5 additions), from an affine Q on the twist, stored in HBM;
//   (2) per event e: M_e = prod over the pairs of line_e(P_i)  (product tree);
//   (3) per batch: Horner over the events, f = (((M_0)^2 M_1 ... )^2 ...) M_67, conj(f).
// (2)+(3) equal blst's shared-squaring miller_loop_n over every pair of the batch.
//
// Lines are scaled by Fp factors (killed by the final exponentiation):
//   line(P) = L0 + (L2 * xP) w^2 + (L3 * yP) w^3   for affine P = (xP, yP).
// The final exponentiation computes the 3rd power of the textbook map (Hayashida-
// Hayasaka-Teruya hard part); the verdict "== 1" is unchanged because gcd(3, r) = 1.
#pragma once
#include "bls_curve.h"

namespace gbls {

struct g2h {  // homogeneous projective point on the twist (x = X/Z, y = Y/Z)
  fp2 x, y, z;
};
struct sp034 {  // sparse Fp12 element a0 + a2 w^2 + a3 w^3
  fp2 a0, a2, a3;
};

// ---------------------------------------------------------------- event schedule
constexpr int ML_EVENTS = 68;
struct ev_mask_t {
  uint64_t lo, hi;
};
constexpr ev_mask_t make_ev_mask() {
  ev_mask_t m{0, 0};
  int e = 0;
  for (int i = 62; i >= 0; i--) {
    if (e < 64)
      m.lo |= 1ull << e;
    else
      m.hi |= 1ull << (e - 64);
    e++;
    if ((k::X_ABS >> i) & 1) e++;
  }
  return m;
}
constexpr ev_mask_t EV_DBL = make_ev_mask();
// event e is a doubling step (f is squared before its line, except at e = 0)
HD bool ev_is_dbl(int e) {
  return e < 64 ? ((EV_DBL.lo >> e) & 1) : ((EV_DBL.hi >> (e - 64)) & 1);
}

// 3 b' a with b' = 4(1 + u): additions only
HD void fp2_mul_3b(fp2 &r, const fp2 &a) {
  fp2 t, s;
  fp2_mul_xi(t, a);
  fp2_add(s, t, t);
  fp2_add(s, s, t);  // 3 (1+u) a
  fp2_add(s, s, s);
  fp2_add(r, s, s);  // 12 (1+u) a
}

// Doubling step on T, line coefficients:  L0 = 3b'Z^2 - Y^2,  L2 = 3X^2,  L3 = -2YZ
HD void line_dbl(g2h &T, fp2 &L0, fp2 &L2, fp2 &L3) {
  fp2 A, B, C, E, F, H, t;
  fp2_mul(A, T.x, T.y);
  fp2_half(A, A);        // XY/2
  fp2_sqr(B, T.y);       // Y^2
  fp2_sqr(C, T.z);       // Z^2
  fp2_add(t, T.y, T.z);
  fp2_sqr(H, t);
  fp2_sub(H, H, B);
  fp2_sub(H, H, C);      // 2YZ
  fp2_mul_3b(E, C);      // 3b'Z^2
  fp2_add(F, E, E);
  fp2_add(F, F, E);      // 3E
  fp2_sub(L0, E, B);
  fp2_sqr(t, T.x);
  fp2_mul3(L2, t);
  fp2_neg(L3, H);
  fp2_sub(t, B, F);
  fp2_mul(T.x, A, t);    // X3 = A (B - F)
  fp2_mul(T.z, B, H);    // Z3 = B H
  fp2_add(t, B, F);
  fp2_half(t, t);
  fp2_sqr(t, t);         // G^2
  fp2_sqr(E, E);
  fp2_mul3(E, E);        // 3E^2
  fp2_sub(T.y, t, E);    // Y3 = G^2 - 3E^2
}

// Addition step T + Q for an affine Q = (x2, y2):
//   theta = Y1 - y2 Z1, lambda = X1 - x2 Z1;  L0 = theta x2 - lambda y2, L2 = -theta,
//   L3 = lambda;  T <- T + Q (homogeneous, add-1998-cmo-2 with Z2 = 1)
HD void line_add_aff(g2h &T, const g2a &Q, fp2 &L0, fp2 &L2, fp2 &L3) {
  fp2 th, la, t;
  fp2_mul(t, Q.y, T.z);
  fp2_sub(th, T.y, t);
  fp2_mul(t, Q.x, T.z);
  fp2_sub(la, T.x, t);
  fp2_mul(L0, th, Q.x);
  fp2_mul(t, la, Q.y);
  fp2_sub(L0, L0, t);
  fp2_neg(L2, th);
  L3 = la;
  fp2 uu, vv, vvv, R, A;
  fp2_sqr(uu, th);
  fp2_sqr(vv, la);
  fp2_mul(vvv, vv, la);
  fp2_neg(vvv, vvv);       // v^3 = -lambda^3
  fp2_mul(R, vv, T.x);
  fp2_mul(A, uu, T.z);
  fp2_sub(A, A, vvv);
  fp2_sub(A, A, R);
  fp2_sub(A, A, R);
  fp2_mul(T.x, la, A);
  fp2_neg(T.x, T.x);       // X3 = v A
  fp2_sub(t, R, A);
  fp2_mul(t, th, t);
  fp2_neg(t, t);           // u (R - A)
  fp2_mul(R, vvv, T.y);
  fp2_sub(T.y, t, R);
  fp2_mul(T.z, vvv, T.z);
}

// A G1 point prepared for line evaluation up to an Fp factor c: for Jacobian (X, Y, Z),
// (x, y, c) = (X Z, Y, Z^3), i.e. x = xP c and y = yP c with c = Z^3; an affine point is
// (x, y, 1) and infinity has c = 0.  The line times c is L0 c + L2 x w^2 + L3 y w^3: the
// Fp factor c is killed by the final exponentiation, so no inversion is needed.
struct g1s {
  fp x, y, c;
};
HD void g1s_from_jac(g1s &r, const g1j &p) {
  if (jac_is_inf(p)) {
    fp_zero(r.x);
    fp_zero(r.y);
    fp_zero(r.c);
    return;
  }
  fp z2;
  fp_sqr(z2, p.z);
  fp_mul(r.c, z2, p.z);
  fp_mul(r.x, p.x, p.z);
  r.y = p.y;
}
HD void g1s_from_aff(g1s &r, const g1a &a) {
  r.x = a.x;
  r.y = a.y;
  if (aff_is_inf(a))
    fp_zero(r.c);
  else
    fp_one(r.c);
}
HD void line_eval_s(sp034 &s, const fp2 &L0, const fp2 &L2, const fp2 &L3, const g1s &P) {
  if (fp_is_zero(P.c)) {
    fp2_one(s.a0);
    fp2_zero(s.a2);
    fp2_zero(s.a3);
    return;
  }
  fp2_mul_fp(s.a0, L0, P.c);
  fp2_mul_fp(s.a2, L2, P.x);
  fp2_mul_fp(s.a3, L3, P.y);
}

// line at an affine G1 point (infinity gives the identity element)
HD void line_eval(sp034 &s, const fp2 &L0, const fp2 &L2, const fp2 &L3, const g1a &P) {
  if (aff_is_inf(P)) {
    fp2_one(s.a0);
    fp2_zero(s.a2);
    fp2_zero(s.a3);
    return;
  }
  s.a0 = L0;
  fp2_mul_fp(s.a2, L2, P.x);
  fp2_mul_fp(s.a3, L3, P.y);
}
HD void sp_to_fp12(fp12 &r, const sp034 &s) {
  r.c0.c0 = s.a0;
  r.c0.c1 = s.a2;  // w^2 = v
  fp2_zero(r.c0.c2);
  fp2_zero(r.c1.c0);
  r.c1.c1 = s.a3;  // w^3 = v w
  fp2_zero(r.c1.c2);
}
// (a0 + a2 w^2 + a3 w^3)(b0 + b2 w^2 + b3 w^3): 6 Fp2 products (Karatsuba pairs; the
// operand sums stay unreduced, fp2_mul takes operands < 2p)
HD void sp_mul_sp(fp12 &r, const sp034 &a, const sp034 &b) {
  fp2 t0, t2, t3, sa, sb, u;
  fp2_mul(t0, a.a0, b.a0);
  fp2_mul(t2, a.a2, b.a2);
  fp2_mul(t3, a.a3, b.a3);
  // w^0: t0 + xi t3
  fp2_mul_xi(u, t3);
  fp2_add(r.c0.c0, t0, u);
  // w^1: 0
  fp2_zero(r.c1.c0);
  // w^2: (a0+a2)(b0+b2) - t0 - t2
  fp2_add_lazy(sa, a.a0, a.a2);
  fp2_add_lazy(sb, b.a0, b.a2);
  fp2_mul(u, sa, sb);
  fp2_sub(u, u, t0);
  fp2_sub(r.c0.c1, u, t2);
  // w^3: (a0+a3)(b0+b3) - t0 - t3
  fp2_add_lazy(sa, a.a0, a.a3);
  fp2_add_lazy(sb, b.a0, b.a3);
  fp2_mul(u, sa, sb);
  fp2_sub(u, u, t0);
  fp2_sub(r.c1.c1, u, t3);
  // w^4: t2
  r.c0.c2 = t2;
  // w^5: (a2+a3)(b2+b3) - t2 - t3
  fp2_add_lazy(sa, a.a2, a.a3);
  fp2_add_lazy(sb, b.a2, b.a3);
  fp2_mul(u, sa, sb);
  fp2_sub(u, u, t2);
  fp2_sub(r.c1.c2, u, t3);
}

// a * (b0 + b1 v): 5 Fp2 products (canonical operands; the Karatsuba operand sums stay
// unreduced, fp2_mul takes operands < 2p)
HD void fp6_mul_01(fp6 &r, const fp6 &a, const fp2 &b0, const fp2 &b1) {
  fp2 t0, t1, s0, s1, c0, c1, c2;
  fp2_mul(t0, a.c0, b0);
  fp2_mul(t1, a.c1, b1);
  fp2_add_lazy(s0, a.c1, a.c2);
  fp2_mul(c0, s0, b1);
  fp2_sub(c0, c0, t1);
  fp2_mul_xi(c0, c0);
  fp2_add(c0, c0, t0);
  fp2_add_lazy(s0, a.c0, a.c1);
  fp2_add_lazy(s1, b0, b1);
  fp2_mul(c1, s0, s1);
  fp2_sub(c1, c1, t0);
  fp2_sub(c1, c1, t1);
  fp2_add_lazy(s0, a.c0, a.c2);
  fp2_mul(c2, s0, b0);
  fp2_sub(c2, c2, t0);
  fp2_add(c2, c2, t1);
  r.c0 = c0;
  r.c1 = c1;
  r.c2 = c2;
}
// a * (b1 v): 3 Fp2 products
HD void fp6_mul_1(fp6 &r, const fp6 &a, const fp2 &b1) {
  fp2 c0, c1, c2;
  fp2_mul(c0, a.c2, b1);
  fp2_mul_xi(c0, c0);
  fp2_mul(c1, a.c0, b1);
  fp2_mul(c2, a.c1, b1);
  r.c0 = c0;
  r.c1 = c1;
  r.c2 = c2;
}
// f * (l0 + l2 w^2 + l3 w^3) = f * ((l0 + l2 v) + (l3 v) w): 13 Fp2 products
HD void fp12_mul_034(fp12 &r, const fp12 &a, const sp034 &s) {
  fp6 t0, t1, u;
  fp6_mul_01(t0, a.c0, s.a0, s.a2);
  fp6_mul_1(t1, a.c1, s.a3);
  fp6_add(u, a.c0, a.c1);
  fp2 l23;
  fp2_add(l23, s.a2, s.a3);
  fp6_mul_01(u, u, s.a0, l23);
  fp6_sub(u, u, t0);
  fp6_sub(r.c1, u, t1);
  fp6_mul_v(t1, t1);
  fp6_add(r.c0, t0, t1);
}

// ---------------------------------------------------------------- line storage (SoA)
// word ((e*6 + c)*12 + limb) * np + pair: one coalesced dword per lane per load
HD size_t line_word(int e, int c, int limb, uint32_t np, uint32_t pair) {
  return (size_t)((e * 6 + c) * 12 + limb) * np + pair;
}
HD void line_put(uint32_t *L, uint32_t np, uint32_t pair, int e, const fp2 &L0, const fp2 &L2,
                 const fp2 &L3) {
  const fp *v[6] = {&L0.c0, &L0.c1, &L2.c0, &L2.c1, &L3.c0, &L3.c1};
#pragma unroll
  for (int c = 0; c < 6; c++)
#pragma unroll
    for (int i = 0; i < 12; i++) L[line_word(e, c, i, np, pair)] = v[c]->l[i];
}
HD void line_get(const uint32_t *L, uint32_t np, uint32_t pair, int e, fp2 &L0, fp2 &L2, fp2 &L3) {
  fp *v[6] = {&L0.c0, &L0.c1, &L2.c0, &L2.c1, &L3.c0, &L3.c1};
#pragma unroll
  for (int c = 0; c < 6; c++)
#pragma unroll
    for (int i = 0; i < 12; i++) v[c]->l[i] = L[line_word(e, c, i, np, pair)];
}
// all 68 lines of Q (identity lines if Q is infinity)
HD void lines_of(uint32_t *L, uint32_t np, uint32_t pair, const g2a &Q) {
  fp2 L0, L2, L3;
  if (aff_is_inf(Q)) {
    fp2_one(L0);
    fp2_zero(L2);
    fp2_zero(L3);
    for (int e = 0; e < ML_EVENTS; e++) line_put(L, np, pair, e, L0, L2, L3);
    return;
  }
  g2h T;
  T.x = Q.x;
  T.y = Q.y;
  fp2_one(T.z);
  int e = 0;
  for (int i = 62; i >= 0; i--) {
    line_dbl(T, L0, L2, L3);
    line_put(L, np, pair, e++, L0, L2, L3);
    if ((k::X_ABS >> i) & 1) {
      line_add_aff(T, Q, L0, L2, L3);
      line_put(L, np, pair, e++, L0, L2, L3);
    }
  }
}

// Lines of events [e0, e1) of Q, stored at event index e - e0 (an event-range slice of
// lines_of).  T carries the running point between slices: read when e0 > 0, written
// when e1 < ML_EVENTS (Ts may be null for the full range).
HD void lines_range(uint32_t *L, uint32_t np, uint32_t pair, const g2a &Q, int e0, int e1, g2h *Ts) {
  fp2 L0, L2, L3;
  if (aff_is_inf(Q)) {
    fp2_one(L0);
    fp2_zero(L2);
    fp2_zero(L3);
    for (int e = e0; e < e1; e++) line_put(L, np, pair, e - e0, L0, L2, L3);
    return;
  }
  g2h T;
  if (e0 > 0) {
    T = Ts[pair];
  } else {
    T.x = Q.x;
    T.y = Q.y;
    fp2_one(T.z);
  }
  for (int e = e0; e < e1; e++) {
    if (ev_is_dbl(e))
      line_dbl(T, L0, L2, L3);
    else
      line_add_aff(T, Q, L0, L2, L3);
    line_put(L, np, pair, e - e0, L0, L2, L3);
  }
  if (e1 < ML_EVENTS) Ts[pair] = T;
}

// Reference single-pair Miller loop (host harness): f_{|x|,Q}(P), conjugated (x < 0).
HD void miller_loop_aff(fp12 &f, const g1a &P, const g2a &Q) {
  fp12_one(f);
  if (aff_is_inf(P) || aff_is_inf(Q)) return;
  g2h T;
  T.x = Q.x;
  T.y = Q.y;
  fp2_one(T.z);
  fp2 L0, L2, L3;
  sp034 s;
  bool first = true;
  for (int i = 62; i >= 0; i--) {
    if (!first) fp12_sqr(f, f);
    line_dbl(T, L0, L2, L3);
    line_eval(s, L0, L2, L3, P);
    if (first)
      sp_to_fp12(f, s);
    else
      fp12_mul_034(f, f, s);
    first = false;
    if ((k::X_ABS >> i) & 1) {
      line_add_aff(T, Q, L0, L2, L3);
      line_eval(s, L0, L2, L3, P);
      fp12_mul_034(f, f, s);
    }
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
// Final exponentiation chain (single lane; the device runs the same chain with the
// wave-cooperative engine, bls_wave12.h):
//   easy: F = f^((p^6-1)(p^2+1));  A = F^(x-1);  A = A^(x-1);  B = A^(x+p);  T = B^x;
//   C = T^x frob2(B) conj(B);  R = C F^3 = f^(3 (p^12-1)/r)
HD void final_exp(fp12 &r, const fp12 &f) {
  fp12 F, A, B, T, t0, t1;
  fp12_inv(t0, f);
  fp12_conj(t1, f);
  fp12_mul(t1, t1, t0);
  fp12_frob2(t0, t1);
  fp12_mul(F, t0, t1);
  fp12_cyc_exp_x(t0, F);
  fp12_conj(t1, F);
  fp12_mul(A, t0, t1);
  fp12_cyc_exp_x(t0, A);
  fp12_conj(t1, A);
  fp12_mul(A, t0, t1);
  fp12_cyc_exp_x(t0, A);
  fp12_frob(t1, A);
  fp12_mul(B, t0, t1);
  fp12_cyc_exp_x(T, B);
  fp12_cyc_exp_x(t0, T);
  fp12_frob2(t1, B);
  fp12_mul(t0, t0, t1);
  fp12_conj(t1, B);
  fp12_mul(t0, t0, t1);
  fp12_sqr(t1, F);
  fp12_mul(t1, t1, F);
  fp12_mul(r, t0, t1);
}

}  // namespace gbls
