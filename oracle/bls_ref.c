/* oracle/bls_ref.c -- TEST INFRASTRUCTURE AND CPU BASELINE ONLY.
 *
 * An independent C restatement of what the reference's signature hot path delegates
 * to blst 0.3.11 (a crates.io dependency, not vendored in /root/reference; SURVEY.md
 * 8(c)): BLS12-381 field tower, G1/G2, RFC 9380 hash_to_G2 (BLS12381G2_XMD:SHA-256_
 * SSWU_RO_), the optimal-ate Miller loop and final exponentiation, and blst's
 * verify_multiple_aggregate_signatures algorithm as called by Signature::multi_verify
 * (bls/src/signature.rs:95-129): per set a 64-bit scalar times pk (G1) and times sig
 * (G2, summed), hash_to_G2, Miller loops in groups of up to 8 pairs sharing the
 * squaring (blst miller_loop_n), per-worker GT products, one merge, one final
 * exponentiation.  Worker threads mirror blst's da_pool.
 *
 * Independence from the GPU engine: 6 x 64-bit limbs (CIOS with 128-bit products)
 * instead of 12 x 32-bit product scanning; Fermat inversion; the Adj-Rodriguez-
 * Henriquez Fp2 square root; the straight RFC 9380 SSWU with inversions; the
 * TEXTBOOK hard part f^((p^4-p^2+1)/r) of the final exponentiation.  Points in the
 * byte API use blst's layout (affine, Montgomery, little-endian 64-bit limbs; all-zero
 * = infinity).  Constants: bls_ref_consts.h (from oracle/bls12_381.py); everything
 * else (R^2, -p^-1, Frobenius/psi coefficients) is derived here at start-up.
 * Not constant time.  Built by oracle/Makefile into oracle/_build/.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef uint64_t u64;
typedef unsigned __int128 u128;
typedef struct { u64 v[6]; } fe;
typedef fe fe_plain;
typedef struct { fe a, b; } fe2; /* a + b u, u^2 = -1 */
typedef fe2 fe2_plain;
typedef struct { fe2 c[3]; } fe6;  /* over v, v^3 = 1 + u */
typedef struct { fe6 c[2]; } fe12; /* over w, w^2 = v */
typedef struct { fe x, y, z; } p1j;
typedef struct { fe x, y; } p1a;
typedef struct { fe2 x, y, z; } p2j;
typedef struct { fe2 x, y; } p2a;

#include "bls_ref_consts.h"

static fe P, ONE, R2, ZERO;
static u64 N0;
static const u64 X_ABS = 0xd201000000010000ull;

/* ------------------------------------------------------------------ Fp */
static int fe_is_zero(const fe *a) { return !(a->v[0] | a->v[1] | a->v[2] | a->v[3] | a->v[4] | a->v[5]); }
static int fe_eq(const fe *a, const fe *b) { return !memcmp(a, b, sizeof(fe)); }
static int geq_p(const u64 *t) {
  for (int i = 5; i >= 0; i--) {
    if (t[i] > P.v[i]) return 1;
    if (t[i] < P.v[i]) return 0;
  }
  return 1;
}
static void sub_p(u64 *t) {
  u64 br = 0;
  for (int i = 0; i < 6; i++) {
    u128 d = (u128)t[i] - P.v[i] - br;
    t[i] = (u64)d;
    br = (u64)(d >> 64) & 1;
  }
}
static void fe_add(fe *r, const fe *a, const fe *b) {
  u64 c = 0;
  for (int i = 0; i < 6; i++) {
    u128 s = (u128)a->v[i] + b->v[i] + c;
    r->v[i] = (u64)s;
    c = (u64)(s >> 64);
  }
  if (geq_p(r->v)) sub_p(r->v);
}
static void fe_sub(fe *r, const fe *a, const fe *b) {
  u64 br = 0;
  for (int i = 0; i < 6; i++) {
    u128 d = (u128)a->v[i] - b->v[i] - br;
    r->v[i] = (u64)d;
    br = (u64)(d >> 64) & 1;
  }
  if (br) {
    u64 c = 0;
    for (int i = 0; i < 6; i++) {
      u128 s = (u128)r->v[i] + P.v[i] + c;
      r->v[i] = (u64)s;
      c = (u64)(s >> 64);
    }
  }
}
static void fe_neg(fe *r, const fe *a) {
  if (fe_is_zero(a)) { *r = *a; return; }
  fe_sub(r, &P, a);  /* P as plain p: p - a */
}
/* CIOS Montgomery product, R = 2^384 */
static void fe_mul(fe *r, const fe *a, const fe *b) {
  u64 t[8] = {0};
  for (int i = 0; i < 6; i++) {
    u128 c = 0;
    for (int j = 0; j < 6; j++) {
      c += (u128)a->v[j] * b->v[i] + t[j];
      t[j] = (u64)c;
      c >>= 64;
    }
    u128 s = (u128)t[6] + (u64)c;
    t[6] = (u64)s;
    t[7] = (u64)(s >> 64);
    u64 m = t[0] * N0;
    c = ((u128)m * P.v[0] + t[0]) >> 64;
    for (int j = 1; j < 6; j++) {
      c += (u128)m * P.v[j] + t[j];
      t[j - 1] = (u64)c;
      c >>= 64;
    }
    s = (u128)t[6] + (u64)c;
    t[5] = (u64)s;
    t[6] = t[7] + (u64)(s >> 64);
  }
  if (t[6] || geq_p(t)) sub_p(t);
  memcpy(r->v, t, 48);
}
static void fe_sqr(fe *r, const fe *a) { fe_mul(r, a, a); }
static void fe_from_plain(fe *r, const fe *a) { fe_mul(r, a, &R2); }
static void fe_to_plain(fe *r, const fe *a) {
  fe one = {{1, 0, 0, 0, 0, 0}};
  fe_mul(r, a, &one);
}
static void fe_from_u64(fe *r, u64 x) {
  fe t = {{x, 0, 0, 0, 0, 0}};
  fe_from_plain(r, &t);
}
/* a^e, e given as 6 little-endian words */
static void fe_pow(fe *r, const fe *a, const u64 *e) {
#ifdef BLS_REF_FAST /* fixed 4-bit windows: 384 squarings + 96 + 14 products */
  fe tab[16];
  tab[0] = ONE;
  tab[1] = *a;
  for (int i = 2; i < 16; i++) fe_mul(&tab[i], &tab[i - 1], a);
  fe acc = ONE;
  for (int i = 380; i >= 0; i -= 4) {
    for (int k = 0; k < 4; k++) fe_sqr(&acc, &acc);
    unsigned d = (unsigned)((e[i >> 6] >> (i & 63)) & 15);
    if (d) fe_mul(&acc, &acc, &tab[d]);
  }
  *r = acc;
#else
  fe acc = ONE;
  for (int i = 383; i >= 0; i--) {
    fe_sqr(&acc, &acc);
    if ((e[i >> 6] >> (i & 63)) & 1) fe_mul(&acc, &acc, a);
  }
  *r = acc;
#endif
}
static u64 E_PM2[6], E_SQRT[6], E_LEG[6], E_PM3D4[6], E_PM1D2[6];
static void fe_inv(fe *r, const fe *a) { fe_pow(r, a, E_PM2); }
static int fe_sqrt(fe *r, const fe *a) {
  fe s, s2;
  fe_pow(&s, a, E_SQRT);
  fe_sqr(&s2, &s);
  *r = s;
  return fe_eq(&s2, a);
}
static int fe_is_square(const fe *a) {
  if (fe_is_zero(a)) return 1;
  fe t;
  fe_pow(&t, a, E_LEG);
  return fe_eq(&t, &ONE);
}
static int fe_sgn0(const fe *a) {
  fe t;
  fe_to_plain(&t, a);
  return (int)(t.v[0] & 1);
}
static int fe_lex_largest(const fe *a) { /* canonical(a) > (p-1)/2 */
  fe t, h;
  fe_to_plain(&t, a);
  for (int i = 0; i < 6; i++) h.v[i] = (P.v[i] >> 1) | (i < 5 ? (P.v[i + 1] << 63) : 0);
  for (int i = 5; i >= 0; i--) {
    if (t.v[i] > h.v[i]) return 1;
    if (t.v[i] < h.v[i]) return 0;
  }
  return 0;
}

/* ------------------------------------------------------------------ Fp2 */
static fe2 F2ONE, F2ZERO;
static int fe2_is_zero(const fe2 *a) { return fe_is_zero(&a->a) && fe_is_zero(&a->b); }
static int fe2_eq(const fe2 *a, const fe2 *b) { return fe_eq(&a->a, &b->a) && fe_eq(&a->b, &b->b); }
static void fe2_add(fe2 *r, const fe2 *a, const fe2 *b) { fe_add(&r->a, &a->a, &b->a); fe_add(&r->b, &a->b, &b->b); }
static void fe2_sub(fe2 *r, const fe2 *a, const fe2 *b) { fe_sub(&r->a, &a->a, &b->a); fe_sub(&r->b, &a->b, &b->b); }
static void fe2_neg(fe2 *r, const fe2 *a) { fe_neg(&r->a, &a->a); fe_neg(&r->b, &a->b); }
static void fe2_conj(fe2 *r, const fe2 *a) { r->a = a->a; fe_neg(&r->b, &a->b); }
#ifdef BLS_REF_FAST /* Karatsuba product (3 Fp products), complex squaring (2) */
static void fe2_mul(fe2 *r, const fe2 *a, const fe2 *b) {
  fe t0, t1, sa, sb;
  fe_mul(&t0, &a->a, &b->a);
  fe_mul(&t1, &a->b, &b->b);
  fe_add(&sa, &a->a, &a->b);
  fe_add(&sb, &b->a, &b->b);
  fe_mul(&sa, &sa, &sb);
  fe_sub(&r->a, &t0, &t1);
  fe_add(&t0, &t0, &t1);
  fe_sub(&r->b, &sa, &t0);
}
static void fe2_sqr(fe2 *r, const fe2 *a) {
  fe s, d, m;
  fe_add(&s, &a->a, &a->b);
  fe_sub(&d, &a->a, &a->b);
  fe_mul(&m, &a->a, &a->b);
  fe_mul(&r->a, &s, &d);
  fe_add(&r->b, &m, &m);
}
#else
static void fe2_mul(fe2 *r, const fe2 *a, const fe2 *b) { /* schoolbook */
  fe t0, t1, t2, t3;
  fe_mul(&t0, &a->a, &b->a);
  fe_mul(&t1, &a->b, &b->b);
  fe_mul(&t2, &a->a, &b->b);
  fe_mul(&t3, &a->b, &b->a);
  fe_sub(&r->a, &t0, &t1);
  fe_add(&r->b, &t2, &t3);
}
static void fe2_sqr(fe2 *r, const fe2 *a) { fe2_mul(r, a, a); }
#endif
static void fe2_mul_fe(fe2 *r, const fe2 *a, const fe *b) { fe_mul(&r->a, &a->a, b); fe_mul(&r->b, &a->b, b); }
static void fe2_mul_xi(fe2 *r, const fe2 *a) { /* (1+u) a */
  fe t0, t1;
  fe_sub(&t0, &a->a, &a->b);
  fe_add(&t1, &a->a, &a->b);
  r->a = t0;
  r->b = t1;
}
static void fe2_inv(fe2 *r, const fe2 *a) {
  fe n, t;
  fe_sqr(&n, &a->a);
  fe_sqr(&t, &a->b);
  fe_add(&n, &n, &t);
  fe_inv(&n, &n);
  fe_mul(&r->a, &a->a, &n);
  fe_mul(&t, &a->b, &n);
  fe_neg(&r->b, &t);
}
static void fe2_pow(fe2 *r, const fe2 *a, const u64 *e) {
#ifdef BLS_REF_FAST /* fixed 4-bit windows */
  fe2 tab[16];
  tab[0] = F2ONE;
  tab[1] = *a;
  for (int i = 2; i < 16; i++) fe2_mul(&tab[i], &tab[i - 1], a);
  fe2 acc = F2ONE;
  for (int i = 380; i >= 0; i -= 4) {
    for (int k = 0; k < 4; k++) fe2_sqr(&acc, &acc);
    unsigned d = (unsigned)((e[i >> 6] >> (i & 63)) & 15);
    if (d) fe2_mul(&acc, &acc, &tab[d]);
  }
  *r = acc;
#else
  fe2 acc = F2ONE;
  for (int i = 383; i >= 0; i--) {
    fe2_sqr(&acc, &acc);
    if ((e[i >> 6] >> (i & 63)) & 1) fe2_mul(&acc, &acc, a);
  }
  *r = acc;
#endif
}
static int fe2_is_square(const fe2 *a) {
  fe n, t;
  fe_sqr(&n, &a->a);
  fe_sqr(&t, &a->b);
  fe_add(&n, &n, &t);
  return fe_is_square(&n);
}
/* Adj & Rodriguez-Henriquez, Alg. 9 (q = p^2, p = 3 mod 4); returns 0 if no root */
static int fe2_sqrt(fe2 *r, const fe2 *a) {
  if (fe2_is_zero(a)) { *r = *a; return 1; }
  fe2 a1, alpha, x0, t, minus1;
  fe2_pow(&a1, a, E_PM3D4);
  fe2_sqr(&t, &a1);
  fe2_mul(&alpha, &t, a);
  fe2_mul(&x0, &a1, a);
  fe2_neg(&minus1, &F2ONE);
  if (fe2_eq(&alpha, &minus1)) { /* x = u x0 */
    fe2 i = {ZERO, ONE};
    fe2_mul(r, &i, &x0);
  } else {
    fe2 b;
    fe2_add(&t, &F2ONE, &alpha);
    fe2_pow(&b, &t, E_PM1D2);
    fe2_mul(r, &b, &x0);
  }
  fe2_sqr(&t, r);
  return fe2_eq(&t, a);
}
static int fe2_sgn0(const fe2 *a) {
  int s0 = fe_sgn0(&a->a), z0 = fe_is_zero(&a->a), s1 = fe_sgn0(&a->b);
  return s0 | (z0 & s1);
}
static int fe2_lex_largest(const fe2 *a) {
  return fe_is_zero(&a->b) ? fe_lex_largest(&a->a) : fe_lex_largest(&a->b);
}

/* ------------------------------------------------------------------ Fp6 / Fp12 */
static void fe6_add(fe6 *r, const fe6 *a, const fe6 *b) { for (int i = 0; i < 3; i++) fe2_add(&r->c[i], &a->c[i], &b->c[i]); }
static void fe6_sub(fe6 *r, const fe6 *a, const fe6 *b) { for (int i = 0; i < 3; i++) fe2_sub(&r->c[i], &a->c[i], &b->c[i]); }
static void fe6_neg(fe6 *r, const fe6 *a) { for (int i = 0; i < 3; i++) fe2_neg(&r->c[i], &a->c[i]); }
static void fe6_mul_v(fe6 *r, const fe6 *a);
#ifdef BLS_REF_FAST /* Karatsuba over Fp2: 6 products, v^3 = xi */
static void fe6_mul(fe6 *r, const fe6 *a, const fe6 *b) {
  fe2 v0, v1, v2, t, u, c0, c1, c2;
  fe2_mul(&v0, &a->c[0], &b->c[0]);
  fe2_mul(&v1, &a->c[1], &b->c[1]);
  fe2_mul(&v2, &a->c[2], &b->c[2]);
  fe2_add(&t, &a->c[1], &a->c[2]); fe2_add(&u, &b->c[1], &b->c[2]); fe2_mul(&t, &t, &u);
  fe2_sub(&t, &t, &v1); fe2_sub(&t, &t, &v2); fe2_mul_xi(&t, &t); fe2_add(&c0, &t, &v0);
  fe2_add(&t, &a->c[0], &a->c[1]); fe2_add(&u, &b->c[0], &b->c[1]); fe2_mul(&t, &t, &u);
  fe2_sub(&t, &t, &v0); fe2_sub(&t, &t, &v1); fe2_mul_xi(&u, &v2); fe2_add(&c1, &t, &u);
  fe2_add(&t, &a->c[0], &a->c[2]); fe2_add(&u, &b->c[0], &b->c[2]); fe2_mul(&t, &t, &u);
  fe2_sub(&t, &t, &v0); fe2_sub(&t, &t, &v2); fe2_add(&c2, &t, &v1);
  r->c[0] = c0; r->c[1] = c1; r->c[2] = c2;
}
#else
static void fe6_mul(fe6 *r, const fe6 *a, const fe6 *b) { /* schoolbook, v^3 = xi */
  fe2 acc[5], t;
  for (int k = 0; k < 5; k++) acc[k] = F2ZERO;
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) {
      fe2_mul(&t, &a->c[i], &b->c[j]);
      fe2_add(&acc[i + j], &acc[i + j], &t);
    }
  fe2_mul_xi(&t, &acc[3]);
  fe2_add(&r->c[0], &acc[0], &t);
  fe2_mul_xi(&t, &acc[4]);
  fe2_add(&r->c[1], &acc[1], &t);
  r->c[2] = acc[2];
}
#endif
static void fe6_mul_v(fe6 *r, const fe6 *a) {
  fe2 t;
  fe2_mul_xi(&t, &a->c[2]);
  r->c[2] = a->c[1];
  r->c[1] = a->c[0];
  r->c[0] = t;
}
static void fe6_inv(fe6 *r, const fe6 *a) {
  fe2 c0, c1, c2, t, s;
  fe2_sqr(&c0, &a->c[0]); fe2_mul(&t, &a->c[1], &a->c[2]); fe2_mul_xi(&t, &t); fe2_sub(&c0, &c0, &t);
  fe2_sqr(&c1, &a->c[2]); fe2_mul_xi(&c1, &c1); fe2_mul(&t, &a->c[0], &a->c[1]); fe2_sub(&c1, &c1, &t);
  fe2_sqr(&c2, &a->c[1]); fe2_mul(&t, &a->c[0], &a->c[2]); fe2_sub(&c2, &c2, &t);
  fe2_mul(&t, &a->c[2], &c1); fe2_mul(&s, &a->c[1], &c2); fe2_add(&t, &t, &s); fe2_mul_xi(&t, &t);
  fe2_mul(&s, &a->c[0], &c0); fe2_add(&t, &t, &s);
  fe2_inv(&t, &t);
  fe2_mul(&r->c[0], &c0, &t); fe2_mul(&r->c[1], &c1, &t); fe2_mul(&r->c[2], &c2, &t);
}
static fe12 F12ONE;
#ifdef BLS_REF_FAST /* Karatsuba over Fp6 (3 products), complex squaring (2 products) */
static void fe12_mul(fe12 *r, const fe12 *a, const fe12 *b) {
  fe6 t0, t1, s, u;
  fe6_mul(&t0, &a->c[0], &b->c[0]);
  fe6_mul(&t1, &a->c[1], &b->c[1]);
  fe6_add(&s, &a->c[0], &a->c[1]);
  fe6_add(&u, &b->c[0], &b->c[1]);
  fe6_mul(&s, &s, &u);
  fe6_sub(&s, &s, &t0);
  fe6_sub(&r->c[1], &s, &t1);
  fe6_mul_v(&t1, &t1);
  fe6_add(&r->c[0], &t0, &t1);
}
static void fe12_sqr(fe12 *r, const fe12 *a) { /* (a0 + a1 w)^2, w^2 = v */
  fe6 m, s, t, u;
  fe6_mul(&m, &a->c[0], &a->c[1]);
  fe6_add(&s, &a->c[0], &a->c[1]);
  fe6_mul_v(&t, &a->c[1]);
  fe6_add(&t, &t, &a->c[0]);
  fe6_mul(&s, &s, &t);          /* (a0 + a1)(a0 + v a1) = a0^2 + v a1^2 + (1 + v) m */
  fe6_sub(&s, &s, &m);
  fe6_mul_v(&u, &m);
  fe6_sub(&r->c[0], &s, &u);    /* a0^2 + v a1^2 */
  fe6_add(&r->c[1], &m, &m);    /* 2 a0 a1 */
}
#else
static void fe12_mul(fe12 *r, const fe12 *a, const fe12 *b) {
  fe6 t0, t1, t2, t3;
  fe6_mul(&t0, &a->c[0], &b->c[0]);
  fe6_mul(&t1, &a->c[1], &b->c[1]);
  fe6_mul(&t2, &a->c[0], &b->c[1]);
  fe6_mul(&t3, &a->c[1], &b->c[0]);
  fe6_mul_v(&t1, &t1);
  fe6_add(&r->c[0], &t0, &t1);
  fe6_add(&r->c[1], &t2, &t3);
}
static void fe12_sqr(fe12 *r, const fe12 *a) { fe12_mul(r, a, a); }
#endif
static void fe12_conj(fe12 *r, const fe12 *a) { r->c[0] = a->c[0]; fe6_neg(&r->c[1], &a->c[1]); }
static void fe12_inv(fe12 *r, const fe12 *a) {
  fe6 t0, t1;
  fe6_mul(&t0, &a->c[0], &a->c[0]);
  fe6_mul(&t1, &a->c[1], &a->c[1]);
  fe6_mul_v(&t1, &t1);
  fe6_sub(&t0, &t0, &t1);
  fe6_inv(&t0, &t0);
  fe6_mul(&r->c[0], &a->c[0], &t0);
  fe6_mul(&t1, &a->c[1], &t0);
  fe6_neg(&r->c[1], &t1);
}
static int fe12_is_one(const fe12 *a) { return !memcmp(a, &F12ONE, sizeof(fe12)); }
/* Frobenius: coefficient of w^e (e = 2j + h) is conj()'d and times GAMMA[e] */
static fe2 GAMMA1[6];
static void fe12_frob(fe12 *r, const fe12 *a) {
  for (int h = 0; h < 2; h++)
    for (int j = 0; j < 3; j++) {
      fe2 t;
      fe2_conj(&t, &a->c[h].c[j]);
      fe2_mul(&r->c[h].c[j], &t, &GAMMA1[2 * j + h]);
    }
}
static void fe12_pow_big(fe12 *r, const fe12 *a, const u64 *e, int nbits) {
  fe12 acc = F12ONE;
  for (int i = nbits - 1; i >= 0; i--) {
    fe12_sqr(&acc, &acc);
    if ((e[i >> 6] >> (i & 63)) & 1) fe12_mul(&acc, &acc, a);
  }
  *r = acc;
}
static u64 E_HARD[24]; /* (p^4 - p^2 + 1) / r: 1269 bits */
static int E_HARD_BITS;
/* textbook final exponentiation: easy part, then f^((p^4-p^2+1)/r) */
static void final_exp(fe12 *r, const fe12 *f) {
  fe12 t0, t1;
  fe12_inv(&t0, f);
  fe12_conj(&t1, f);
  fe12_mul(&t1, &t1, &t0);  /* f^(p^6-1) */
  fe12_frob(&t0, &t1);
  fe12_frob(&t0, &t0);
  fe12_mul(&t1, &t0, &t1);  /* ^(p^2+1) */
  fe12_pow_big(r, &t1, E_HARD, E_HARD_BITS);
}

/* ------------------------------------------------------------------ curves (Jacobian) */
#define DEF_CURVE(PFX, F, PJ, PA, ADD, SUB, MUL, SQR, NEG, ISZ, EQ, ONEV, ZEROV)          \
  static int PFX##_is_inf(const PJ *p) { return ISZ(&p->z); }                            \
  static int PFX##a_is_inf(const PA *p) { return ISZ(&p->x) && ISZ(&p->y); }             \
  static void PFX##_set_inf(PJ *r) { r->x = ONEV; r->y = ONEV; r->z = ZEROV; }           \
  static void PFX##_from_aff(PJ *r, const PA *a) {                                       \
    r->x = a->x; r->y = a->y;                                                            \
    if (PFX##a_is_inf(a)) r->z = ZEROV; else r->z = ONEV;                                \
  }                                                                                      \
  static void PFX##_dbl(PJ *r, const PJ *p) {                                            \
    if (PFX##_is_inf(p)) { *r = *p; return; }                                            \
    F A, B, C, D, E, G, t;                                                               \
    SQR(&A, &p->x); SQR(&B, &p->y); SQR(&C, &B);                                         \
    ADD(&t, &p->x, &B); SQR(&t, &t); SUB(&t, &t, &A); SUB(&t, &t, &C); ADD(&D, &t, &t);   \
    ADD(&E, &A, &A); ADD(&E, &E, &A); SQR(&G, &E);                                       \
    PJ o;                                                                                \
    MUL(&t, &p->y, &p->z); ADD(&o.z, &t, &t);                                            \
    SUB(&o.x, &G, &D); SUB(&o.x, &o.x, &D);                                              \
    SUB(&t, &D, &o.x); MUL(&t, &E, &t);                                                  \
    ADD(&C, &C, &C); ADD(&C, &C, &C); ADD(&C, &C, &C); SUB(&o.y, &t, &C);                \
    *r = o;                                                                              \
  }                                                                                      \
  static void PFX##_add(PJ *r, const PJ *p, const PJ *q) {                               \
    if (PFX##_is_inf(p)) { *r = *q; return; }                                            \
    if (PFX##_is_inf(q)) { *r = *p; return; }                                            \
    F z1z1, z2z2, u1, u2, s1, s2, h, i, j, rr, v, t;                                     \
    SQR(&z1z1, &p->z); SQR(&z2z2, &q->z);                                                \
    MUL(&u1, &p->x, &z2z2); MUL(&u2, &q->x, &z1z1);                                      \
    MUL(&s1, &p->y, &q->z); MUL(&s1, &s1, &z2z2);                                        \
    MUL(&s2, &q->y, &p->z); MUL(&s2, &s2, &z1z1);                                        \
    SUB(&h, &u2, &u1); SUB(&rr, &s2, &s1);                                               \
    if (ISZ(&h)) {                                                                       \
      if (ISZ(&rr)) PFX##_dbl(r, p); else PFX##_set_inf(r);                              \
      return;                                                                            \
    }                                                                                    \
    ADD(&i, &h, &h); SQR(&i, &i); MUL(&j, &h, &i); ADD(&rr, &rr, &rr); MUL(&v, &u1, &i); \
    PJ o;                                                                                \
    SQR(&o.x, &rr); SUB(&o.x, &o.x, &j); SUB(&o.x, &o.x, &v); SUB(&o.x, &o.x, &v);       \
    SUB(&t, &v, &o.x); MUL(&t, &rr, &t); MUL(&s1, &s1, &j); ADD(&s1, &s1, &s1);          \
    SUB(&o.y, &t, &s1);                                                                  \
    ADD(&t, &p->z, &q->z); SQR(&t, &t); SUB(&t, &t, &z1z1); SUB(&t, &t, &z2z2);          \
    MUL(&o.z, &t, &h);                                                                   \
    *r = o;                                                                              \
  }                                                                                      \
  static void PFX##_add_aff(PJ *r, const PJ *p, const PA *q) {                           \
    PJ qj;                                                                               \
    PFX##_from_aff(&qj, q);                                                              \
    PFX##_add(r, p, &qj);                                                                \
  }                                                                                      \
  static void PFX##_neg(PJ *r, const PJ *p) { r->x = p->x; NEG(&r->y, &p->y); r->z = p->z; } \
  static void PFX##_mul_u64(PJ *r, const PA *b, u64 k) {                                 \
    PJ acc;                                                                              \
    PFX##_set_inf(&acc);                                                                 \
    for (int i = 63; i >= 0; i--) {                                                      \
      PFX##_dbl(&acc, &acc);                                                             \
      if ((k >> i) & 1) PFX##_add_aff(&acc, &acc, b);                                    \
    }                                                                                    \
    *r = acc;                                                                            \
  }                                                                                      \
  static void PFX##_mul_words(PJ *r, const PJ *b, const u64 *k, int nbits) {             \
    PJ acc;                                                                              \
    PFX##_set_inf(&acc);                                                                 \
    for (int i = nbits - 1; i >= 0; i--) {                                               \
      PFX##_dbl(&acc, &acc);                                                             \
      if ((k[i >> 6] >> (i & 63)) & 1) PFX##_add(&acc, &acc, b);                         \
    }                                                                                    \
    *r = acc;                                                                            \
  }

DEF_CURVE(p1, fe, p1j, p1a, fe_add, fe_sub, fe_mul, fe_sqr, fe_neg, fe_is_zero, fe_eq, ONE, ZERO)
DEF_CURVE(p2, fe2, p2j, p2a, fe2_add, fe2_sub, fe2_mul, fe2_sqr, fe2_neg, fe2_is_zero, fe2_eq, F2ONE, F2ZERO)

static void p1_to_aff(p1a *r, const p1j *p) {
  if (p1_is_inf(p)) { r->x = ZERO; r->y = ZERO; return; }
  fe zi, z2, z3;
  fe_inv(&zi, &p->z); fe_sqr(&z2, &zi); fe_mul(&z3, &z2, &zi);
  fe_mul(&r->x, &p->x, &z2); fe_mul(&r->y, &p->y, &z3);
}
static void p2_to_aff(p2a *r, const p2j *p) {
  if (p2_is_inf(p)) { r->x = F2ZERO; r->y = F2ZERO; return; }
  fe2 zi, z2, z3;
  fe2_inv(&zi, &p->z); fe2_sqr(&z2, &zi); fe2_mul(&z3, &z2, &zi);
  fe2_mul(&r->x, &p->x, &z2); fe2_mul(&r->y, &p->y, &z3);
}
static fe2 PSI_CX, PSI_CY, B2;
static fe B1;
static void p2_psi(p2j *r, const p2j *p) { /* psi on Jacobian coordinates (z conjugated) */
  fe2 t;
  fe2_conj(&t, &p->x); fe2_mul(&r->x, &t, &PSI_CX);
  fe2_conj(&t, &p->y); fe2_mul(&r->y, &t, &PSI_CY);
  fe2_conj(&r->z, &p->z);
}
static u64 R_ORDER[4];
static int p2_in_group(const p2a *a) { /* [r] P == O */
  if (p2a_is_inf(a)) return 1;
  p2j p, t;
  p2_from_aff(&p, a);
  p2_mul_words(&t, &p, R_ORDER, 255);
  return p2_is_inf(&t);
}
static int p2_on_curve(const p2a *a) {
  fe2 l, r;
  fe2_sqr(&l, &a->y); fe2_sqr(&r, &a->x); fe2_mul(&r, &r, &a->x); fe2_add(&r, &r, &B2);
  return fe2_eq(&l, &r);
}

/* ------------------------------------------------------------------ SHA-256 */
static const uint32_t K256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};
#define ROR(x, n) (((x) >> (n)) | ((x) << (32 - (n))))
static void sha256(const uint8_t *msg, size_t len, uint8_t out[32]) {
  uint32_t h[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  size_t total = ((len + 9 + 63) / 64) * 64;
  uint8_t *buf = calloc(total, 1);
  memcpy(buf, msg, len);
  buf[len] = 0x80;
  uint64_t bits = (uint64_t)len * 8;
  for (int i = 0; i < 8; i++) buf[total - 1 - i] = (uint8_t)(bits >> (8 * i));
  for (size_t off = 0; off < total; off += 64) {
    uint32_t w[64];
    for (int i = 0; i < 16; i++)
      w[i] = ((uint32_t)buf[off + 4 * i] << 24) | ((uint32_t)buf[off + 4 * i + 1] << 16) |
             ((uint32_t)buf[off + 4 * i + 2] << 8) | buf[off + 4 * i + 3];
    for (int i = 16; i < 64; i++) {
      uint32_t s0 = ROR(w[i - 15], 7) ^ ROR(w[i - 15], 18) ^ (w[i - 15] >> 3);
      uint32_t s1 = ROR(w[i - 2], 17) ^ ROR(w[i - 2], 19) ^ (w[i - 2] >> 10);
      w[i] = w[i - 16] + s0 + w[i - 7] + s1;
    }
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
    for (int i = 0; i < 64; i++) {
      uint32_t t1 = hh + (ROR(e, 6) ^ ROR(e, 11) ^ ROR(e, 25)) + ((e & f) ^ (~e & g)) + K256[i] + w[i];
      uint32_t t2 = (ROR(a, 2) ^ ROR(a, 13) ^ ROR(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
      hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
  }
  free(buf);
  for (int i = 0; i < 8; i++)
    for (int k = 0; k < 4; k++) out[4 * i + k] = (uint8_t)(h[i] >> (24 - 8 * k));
}

/* ------------------------------------------------------------------ hash_to_G2 (RFC 9380) */
static void expand_message_xmd(const uint8_t *msg, size_t mlen, const uint8_t *dst, size_t dlen,
                               uint8_t *out, size_t outlen) {
  size_t ell = (outlen + 31) / 32;
  uint8_t *b0in = calloc(64 + mlen + 3 + dlen + 1, 1);
  memcpy(b0in + 64, msg, mlen);
  b0in[64 + mlen] = (uint8_t)(outlen >> 8);
  b0in[64 + mlen + 1] = (uint8_t)outlen;
  b0in[64 + mlen + 2] = 0;
  memcpy(b0in + 64 + mlen + 3, dst, dlen);
  b0in[64 + mlen + 3 + dlen] = (uint8_t)dlen;
  uint8_t b0[32], bi[32], in[32 + 1 + 256];
  sha256(b0in, 64 + mlen + 3 + dlen + 1, b0);
  free(b0in);
  memcpy(in, b0, 32);
  for (size_t i = 1; i <= ell; i++) {
    if (i > 1)
      for (int k = 0; k < 32; k++) in[k] = b0[k] ^ bi[k];
    in[32] = (uint8_t)i;
    memcpy(in + 33, dst, dlen);
    in[33 + dlen] = (uint8_t)dlen;
    sha256(in, 34 + dlen, bi);
    memcpy(out + 32 * (i - 1), bi, (32 * i <= outlen) ? 32 : outlen - 32 * (i - 1));
  }
}
static fe F2_256; /* 2^256 in Montgomery form */
static void fe_from_be64(fe *r, const uint8_t *b) { /* 64 big-endian bytes mod p */
  fe hi = {{0}}, lo = {{0}};
  for (int i = 0; i < 32; i++) {
    hi.v[i / 8] |= (u64)b[31 - i] << (8 * (i % 8));
    lo.v[i / 8] |= (u64)b[63 - i] << (8 * (i % 8));
  }
  fe h, l;
  fe_from_plain(&h, &hi);
  fe_from_plain(&l, &lo);
  fe_mul(&h, &h, &F2_256);
  fe_add(r, &h, &l);
}
static fe2 SSWU_A, SSWU_B, SSWU_Z, ISO_XNUM[4], ISO_XDEN[3], ISO_YNUM[4], ISO_YDEN[4];
static void map_to_curve_sswu(p2a *r, const fe2 *u) { /* RFC 9380 6.6.2, straight line */
  fe2 u2, tv1, x1, gx1, x, y, t, t2;
  fe2_sqr(&u2, u);
  fe2_mul(&t, &SSWU_Z, &u2);             /* Z u^2 */
  fe2_sqr(&tv1, &t);
  fe2_add(&tv1, &tv1, &t);               /* Z^2 u^4 + Z u^2 */
  if (fe2_is_zero(&tv1)) {               /* x1 = B / (Z A) */
    fe2_mul(&t2, &SSWU_Z, &SSWU_A);
    fe2_inv(&t2, &t2);
    fe2_mul(&x1, &SSWU_B, &t2);
  } else {                               /* x1 = (-B / A) (1 + 1/tv1) */
    fe2_inv(&t2, &tv1);
    fe2_add(&t2, &t2, &F2ONE);
    fe2 nb, ai;
    fe2_neg(&nb, &SSWU_B);
    fe2_inv(&ai, &SSWU_A);
    fe2_mul(&nb, &nb, &ai);
    fe2_mul(&x1, &nb, &t2);
  }
  fe2_sqr(&gx1, &x1); fe2_add(&gx1, &gx1, &SSWU_A); fe2_mul(&gx1, &gx1, &x1); fe2_add(&gx1, &gx1, &SSWU_B);
  if (fe2_is_square(&gx1)) {
    x = x1;
    fe2_sqrt(&y, &gx1);
  } else {
    fe2 gx2;
    fe2_mul(&x, &t, &x1);                /* Z u^2 x1 */
    fe2_sqr(&gx2, &x); fe2_add(&gx2, &gx2, &SSWU_A); fe2_mul(&gx2, &gx2, &x); fe2_add(&gx2, &gx2, &SSWU_B);
    fe2_sqrt(&y, &gx2);
  }
  if (fe2_sgn0(u) != fe2_sgn0(&y)) fe2_neg(&y, &y);
  r->x = x;
  r->y = y;
}
static void poly(fe2 *r, const fe2 *c, int n, const fe2 *x) { /* sum c_i x^i (Horner) */
  fe2 acc = c[n - 1];
  for (int i = n - 2; i >= 0; i--) { fe2_mul(&acc, &acc, x); fe2_add(&acc, &acc, &c[i]); }
  *r = acc;
}
static void iso_map(p2j *r, const p2a *p) {
  fe2 xn, xd, yn, yd, t;
  poly(&xn, ISO_XNUM, 4, &p->x); poly(&xd, ISO_XDEN, 3, &p->x);
  poly(&yn, ISO_YNUM, 4, &p->x); poly(&yd, ISO_YDEN, 4, &p->x);
  if (fe2_is_zero(&xd) || fe2_is_zero(&yd)) { p2_set_inf(r); return; }
  p2a a;
  fe2_inv(&t, &xd); fe2_mul(&a.x, &xn, &t);
  fe2_inv(&t, &yd); fe2_mul(&t, &yn, &t); fe2_mul(&a.y, &p->y, &t);
  p2_from_aff(r, &a);
}
static void mul_by_x(p2j *r, const p2j *p) { /* [x]P, x < 0 */
  u64 k = X_ABS;
  p2_mul_words(r, p, &k, 64);
  p2_neg(r, r);
}
static void clear_cofactor(p2j *r, const p2j *p) { /* Budroni-Pintore */
  p2j t1, t2, t3, s;
  mul_by_x(&t1, p);
  p2_psi(&t2, p);
  p2_dbl(&t3, p);
  p2_psi(&t3, &t3);
  p2_psi(&t3, &t3);
  p2_neg(&s, &t2);
  p2_add(&t3, &t3, &s);
  p2_add(&t2, &t1, &t2);
  mul_by_x(&t2, &t2);
  p2_add(&t3, &t3, &t2);
  p2_neg(&s, &t1);
  p2_add(&t3, &t3, &s);
  p2_neg(&s, p);
  p2_add(r, &t3, &s);
}
static const uint8_t DST_POP[] = "BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_";
static void hash_to_g2(p2a *out, const uint8_t *msg, size_t len, const uint8_t *dst, size_t dlen) {
  uint8_t u[256];
  expand_message_xmd(msg, len, dst, dlen, u, 256);
  fe2 e0, e1;
  fe_from_be64(&e0.a, u); fe_from_be64(&e0.b, u + 64);
  fe_from_be64(&e1.a, u + 128); fe_from_be64(&e1.b, u + 192);
  p2a q0, q1;
  map_to_curve_sswu(&q0, &e0);
  map_to_curve_sswu(&q1, &e1);
  p2j a, b, h;
  iso_map(&a, &q0);
  iso_map(&b, &q1);
  p2_add(&a, &a, &b);
  clear_cofactor(&h, &a);
  p2_to_aff(out, &h);
}

/* ------------------------------------------------------------------ pairing */
typedef struct { fe2 x, y, z; } p2h; /* homogeneous projective point on the twist */
typedef struct { fe2 a0, a2, a3; } line_t; /* a0 + a2 xP w^2 + a3 yP w^3 */
static fe INV2;
static fe2 B3; /* 3 b' */
/* doubling step (Costello-Lange-Naehrig, y^2 = x^3 + b'): line 3b'Z^2 - Y^2, 3X^2, -2YZ */
static void line_dbl(p2h *T, line_t *l) {
  fe2 A, B, C, E, F, G, H, t, t3;
  fe2_mul(&A, &T->x, &T->y); fe2_mul_fe(&A, &A, &INV2);
  fe2_sqr(&B, &T->y); fe2_sqr(&C, &T->z);
  fe2_mul(&E, &B3, &C);
  fe2_add(&F, &E, &E); fe2_add(&F, &F, &E);
  fe2_add(&t, &T->y, &T->z); fe2_sqr(&H, &t); fe2_sub(&H, &H, &B); fe2_sub(&H, &H, &C);
  fe2_sub(&l->a0, &E, &B);
  fe2_sqr(&t, &T->x); fe2_add(&l->a2, &t, &t); fe2_add(&l->a2, &l->a2, &t);
  fe2_neg(&l->a3, &H);
  fe2_sub(&t, &B, &F); fe2_mul(&T->x, &A, &t);
  fe2_add(&G, &B, &F); fe2_mul_fe(&G, &G, &INV2); fe2_sqr(&G, &G);
  fe2_sqr(&t, &E); fe2_add(&t3, &t, &t); fe2_add(&t3, &t3, &t);
  fe2_sub(&T->y, &G, &t3);
  fe2_mul(&T->z, &B, &H);
}
/* mixed addition step T + Q (Q affine): line theta x2 - lambda y2, -theta, lambda */
static void line_add(p2h *T, const p2a *Q, line_t *l) {
  fe2 th, la, t, uu, vv, vvv, R, A;
  fe2_mul(&t, &Q->y, &T->z); fe2_sub(&th, &T->y, &t);
  fe2_mul(&t, &Q->x, &T->z); fe2_sub(&la, &T->x, &t);
  fe2_mul(&l->a0, &th, &Q->x); fe2_mul(&t, &la, &Q->y); fe2_sub(&l->a0, &l->a0, &t);
  fe2_neg(&l->a2, &th);
  l->a3 = la;
  fe2_sqr(&uu, &th); fe2_sqr(&vv, &la); fe2_mul(&vvv, &vv, &la); fe2_neg(&vvv, &vvv);
  fe2_mul(&R, &vv, &T->x);
  fe2_mul(&A, &uu, &T->z); fe2_sub(&A, &A, &vvv); fe2_sub(&A, &A, &R); fe2_sub(&A, &A, &R);
  fe2_mul(&T->x, &la, &A); fe2_neg(&T->x, &T->x);
  fe2_sub(&t, &R, &A); fe2_mul(&t, &th, &t); fe2_neg(&t, &t);
  fe2_mul(&R, &vvv, &T->y); fe2_sub(&T->y, &t, &R);
  fe2_mul(&T->z, &vvv, &T->z);
}
/* f *= (b0 + b1 v) + (c v) w  with b0 = a0, b1 = a2 xP, c = a3 yP  (w^2 = v, v^3 = xi) */
static void mul_by_line(fe12 *f, const line_t *l, const p1a *P) {
  fe2 b0 = l->a0, b1, c, u;
  fe2_mul_fe(&b1, &l->a2, &P->x);
  fe2_mul_fe(&c, &l->a3, &P->y);
  const fe6 *x = &f->c[0], *y = &f->c[1];
  fe6 xb, yb, ycv2, xcv;
  /* x (b0 + b1 v), y (b0 + b1 v) */
  fe2_mul(&xb.c[0], &x->c[0], &b0); fe2_mul(&u, &x->c[2], &b1); fe2_mul_xi(&u, &u); fe2_add(&xb.c[0], &xb.c[0], &u);
  fe2_mul(&xb.c[1], &x->c[0], &b1); fe2_mul(&u, &x->c[1], &b0); fe2_add(&xb.c[1], &xb.c[1], &u);
  fe2_mul(&xb.c[2], &x->c[1], &b1); fe2_mul(&u, &x->c[2], &b0); fe2_add(&xb.c[2], &xb.c[2], &u);
  fe2_mul(&yb.c[0], &y->c[0], &b0); fe2_mul(&u, &y->c[2], &b1); fe2_mul_xi(&u, &u); fe2_add(&yb.c[0], &yb.c[0], &u);
  fe2_mul(&yb.c[1], &y->c[0], &b1); fe2_mul(&u, &y->c[1], &b0); fe2_add(&yb.c[1], &yb.c[1], &u);
  fe2_mul(&yb.c[2], &y->c[1], &b1); fe2_mul(&u, &y->c[2], &b0); fe2_add(&yb.c[2], &yb.c[2], &u);
  /* y (c v) w^2 = y c v^2: (y0 + y1 v + y2 v^2) c v^2 = xi y1 c + xi y2 c v + y0 c v^2 */
  fe2_mul(&u, &y->c[1], &c); fe2_mul_xi(&ycv2.c[0], &u);
  fe2_mul(&u, &y->c[2], &c); fe2_mul_xi(&ycv2.c[1], &u);
  fe2_mul(&ycv2.c[2], &y->c[0], &c);
  /* x (c v) = xi x2 c + x0 c v + x1 c v^2 */
  fe2_mul(&u, &x->c[2], &c); fe2_mul_xi(&xcv.c[0], &u);
  fe2_mul(&xcv.c[1], &x->c[0], &c);
  fe2_mul(&xcv.c[2], &x->c[1], &c);
  fe6_add(&f->c[0], &xb, &ycv2);
  fe6_add(&f->c[1], &yb, &xcv);
}
/* prod_k f_{|x|,Q_k}(P_k) with one shared squaring per step (blst miller_loop_n),
 * conjugated (x < 0) */
static void miller_loop_n(fe12 *f, const p1a *P, const p2a *Q, int n) {
  p2h T[8];
  line_t l;
  *f = F12ONE;
  for (int k = 0; k < n; k++) { T[k].x = Q[k].x; T[k].y = Q[k].y; T[k].z = F2ONE; }
  int first = 1;
  for (int i = 62; i >= 0; i--) {
    if (!first) fe12_sqr(f, f);
    first = 0;
    for (int k = 0; k < n; k++) { line_dbl(&T[k], &l); mul_by_line(f, &l, &P[k]); }
    if ((X_ABS >> i) & 1)
      for (int k = 0; k < n; k++) { line_add(&T[k], &Q[k], &l); mul_by_line(f, &l, &P[k]); }
  }
  fe12_conj(f, f);
}

/* ------------------------------------------------------------------ initialisation */
static p1a G1;
static p2a G2;
static void from_plain2(fe2 *r, const fe2_plain *a) { fe_from_plain(&r->a, &a->a); fe_from_plain(&r->b, &a->b); }
static void w_sub_small(u64 *r, const u64 *a, u64 s) {
  u64 br = s;
  for (int i = 0; i < 6; i++) { u128 d = (u128)a[i] - br; r[i] = (u64)d; br = (u64)(d >> 64) & 1; }
}
static void w_add_small(u64 *r, const u64 *a, u64 s) {
  u64 c = s;
  for (int i = 0; i < 6; i++) { u128 t = (u128)a[i] + c; r[i] = (u64)t; c = (u64)(t >> 64); }
}
static void w_shr(u64 *r, const u64 *a, int k) {
  for (int i = 0; i < 6; i++) r[i] = (a[i] >> k) | (i < 5 ? a[i + 1] << (64 - k) : 0);
}
static void w_div_small(u64 *r, const u64 *a, u64 d) {
  u128 rem = 0;
  for (int i = 5; i >= 0; i--) { u128 cur = (rem << 64) | a[i]; r[i] = (u64)(cur / d); rem = cur % d; }
}
static void init_once(void) {
  P = C_P;
  memset(&ZERO, 0, sizeof ZERO);
  u64 inv = 1;
  for (int i = 0; i < 7; i++) inv *= 2 - P.v[0] * inv;
  N0 = (u64)0 - inv;
  fe x = {{1, 0, 0, 0, 0, 0}};
  for (int i = 0; i < 768; i++) fe_add(&x, &x, &x); /* 2^768 mod p (plain) */
  R2 = x;
  fe_from_u64(&ONE, 1);
  w_sub_small(E_PM2, P.v, 2);
  w_add_small(E_SQRT, P.v, 1); w_shr(E_SQRT, E_SQRT, 2);
  w_sub_small(E_LEG, P.v, 1); w_shr(E_LEG, E_LEG, 1);
  w_sub_small(E_PM3D4, P.v, 3); w_shr(E_PM3D4, E_PM3D4, 2);
  memcpy(E_PM1D2, E_LEG, sizeof E_LEG);
  F2ONE.a = ONE; F2ONE.b = ZERO;
  F2ZERO.a = ZERO; F2ZERO.b = ZERO;
  memset(&F12ONE, 0, sizeof F12ONE);
  F12ONE.c[0].c[0] = F2ONE;
  fe_from_u64(&B1, 4);
  B2.a = B1; B2.b = B1;
  fe2_add(&B3, &B2, &B2); fe2_add(&B3, &B3, &B2);
  fe two;
  fe_from_u64(&two, 2);
  fe_inv(&INV2, &two);
  fe p256 = {{0, 0, 0, 0, 1, 0}};
  fe_from_plain(&F2_256, &p256);
  from_plain2(&SSWU_A, &C_SSWU_A); from_plain2(&SSWU_B, &C_SSWU_B); from_plain2(&SSWU_Z, &C_SSWU_Z);
  for (int i = 0; i < 4; i++) {
    from_plain2(&ISO_XNUM[i], &C_ISO_XNUM[i]);
    from_plain2(&ISO_YNUM[i], &C_ISO_YNUM[i]);
    from_plain2(&ISO_YDEN[i], &C_ISO_YDEN[i]);
  }
  for (int i = 0; i < 3; i++) from_plain2(&ISO_XDEN[i], &C_ISO_XDEN[i]);
  fe_from_plain(&G1.x, &C_G1X); fe_from_plain(&G1.y, &C_G1Y);
  from_plain2(&G2.x, &C_G2X); from_plain2(&G2.y, &C_G2Y);
  u64 e6[6], pm1[6];
  w_sub_small(pm1, P.v, 1);
  w_div_small(e6, pm1, 6);
  fe2 xi = {ONE, ONE}, g1;
  fe2_pow(&g1, &xi, e6); /* xi^((p-1)/6) */
  GAMMA1[0] = F2ONE;
  for (int e = 1; e < 6; e++) fe2_mul(&GAMMA1[e], &GAMMA1[e - 1], &g1);
  fe2_inv(&PSI_CX, &GAMMA1[2]); /* 1 / xi^((p-1)/3) */
  fe2_inv(&PSI_CY, &GAMMA1[3]); /* 1 / xi^((p-1)/2) */
  memcpy(E_HARD, C_E_HARD, sizeof C_E_HARD);
  E_HARD_BITS = C_E_HARD_BITS;
  memcpy(R_ORDER, C_R, sizeof C_R);
}
static pthread_once_t g_once = PTHREAD_ONCE_INIT;
static void ensure_init(void) { pthread_once(&g_once, init_once); }

/* ------------------------------------------------------------------ exported API */
typedef struct {
  const uint8_t *msgs, *sigs, *pks;
  const u64 *rands;
  size_t b, e;
  fe12 f;
  p2j S;
  int bad;
} job_t;
static void *mv_worker(void *arg) {
  job_t *j = (job_t *)arg;
  j->f = F12ONE;
  p2_set_inf(&j->S);
  j->bad = 0;
  p1a Pg[8];
  p2a Qg[8];
  int ng = 0;
  for (size_t i = j->b; i < j->e; i++) {
    p1a pk;
    p2a sig;
    memcpy(&pk, j->pks + 96 * i, 96);
    memcpy(&sig, j->sigs + 192 * i, 192);
    if (p1a_is_inf(&pk)) { j->bad = 1; continue; } /* blst: PAIRING_Aggregate_PK_in_G1 */
    u64 r = j->rands[i];
    p2a H;
    hash_to_g2(&H, j->msgs + 32 * i, 32, DST_POP, 43);
    p1j t;
    p1_mul_u64(&t, &pk, r);
    p1_to_aff(&Pg[ng], &t);
    if (!p2a_is_inf(&sig)) { /* infinite signatures are skipped in the sum */
      p2j R;
      p2_mul_u64(&R, &sig, r);
      p2_add(&j->S, &j->S, &R);
    }
    Qg[ng++] = H;
    if (ng == 8) {
      fe12 g;
      miller_loop_n(&g, Pg, Qg, ng);
      fe12_mul(&j->f, &j->f, &g);
      ng = 0;
    }
  }
  if (ng) {
    fe12 g;
    miller_loop_n(&g, Pg, Qg, ng);
    fe12_mul(&j->f, &j->f, &g);
  }
  return NULL;
}
/* Signature::multi_verify with caller-supplied nonzero 64-bit scalars: 1 = valid */
int ref_multi_verify(const uint8_t *msgs32, const uint8_t *sigs192, const uint8_t *pks96, const uint64_t *rands,
                     size_t n, int nthreads) {
  ensure_init();
  if (n == 0) return 0;
  if (nthreads < 1) nthreads = 1;
  if ((size_t)nthreads > n) nthreads = (int)n;
  job_t *jobs = calloc(nthreads, sizeof(job_t));
  pthread_t *th = calloc(nthreads, sizeof(pthread_t));
  for (int t = 0; t < nthreads; t++) {
    jobs[t].msgs = msgs32; jobs[t].sigs = sigs192; jobs[t].pks = pks96; jobs[t].rands = rands;
    jobs[t].b = n * t / nthreads; jobs[t].e = n * (t + 1) / nthreads;
    pthread_create(&th[t], NULL, mv_worker, &jobs[t]);
  }
  fe12 f = F12ONE;
  p2j S;
  p2_set_inf(&S);
  int bad = 0;
  for (int t = 0; t < nthreads; t++) {
    pthread_join(th[t], NULL);
    fe12_mul(&f, &f, &jobs[t].f);
    p2_add(&S, &S, &jobs[t].S);
    bad |= jobs[t].bad;
  }
  free(jobs);
  free(th);
  if (bad) return 0;
  if (!p2_is_inf(&S)) {
    p2a Sa;
    p2_to_aff(&Sa, &S);
    p1a ng1 = G1;
    fe_neg(&ng1.y, &ng1.y);
    fe12 g;
    miller_loop_n(&g, &ng1, &Sa, 1);
    fe12_mul(&f, &f, &g);
  }
  fe12 r;
  final_exp(&r, &f);
  return fe12_is_one(&r);
}
/* Sharded multi_verify: one shard's Miller partial
   F = prod_i ML(r_i pk_i, H(m_i)) * ML(-g1, sum_i r_i sig_i), no final exponentiation.
   Returns the shard's error flag (an infinite pk). out576 = the Fp12 partial. */
int ref_multi_verify_partial(const uint8_t *msgs32, const uint8_t *sigs192, const uint8_t *pks96,
                             const uint64_t *rands, size_t n, uint8_t *out576) {
  ensure_init();
  job_t job;
  memset(&job, 0, sizeof job);
  job.msgs = msgs32; job.sigs = sigs192; job.pks = pks96; job.rands = rands;
  job.b = 0; job.e = n;
  fe12 f = F12ONE;
  int bad = 0;
  if (n) {
    mv_worker(&job);
    f = job.f;
    bad = job.bad;
    if (!p2_is_inf(&job.S)) {
      p2a Sa;
      p2_to_aff(&Sa, &job.S);
      p1a ng1 = G1;
      fe_neg(&ng1.y, &ng1.y);
      fe12 g;
      miller_loop_n(&g, &ng1, &Sa, 1);
      fe12_mul(&f, &f, &g);
    }
  }
  memcpy(out576, &f, sizeof f);
  return bad;
}
/* product of nparts shard partials, final exponentiation, verdict: 1 = valid */
int ref_final_verify_partials(const uint8_t *parts576, const int32_t *errs, size_t nparts) {
  ensure_init();
  fe12 f = F12ONE, g;
  for (size_t k = 0; k < nparts; k++) {
    if (errs[k]) return 0;
    memcpy(&g, parts576 + 576 * k, 576);
    fe12_mul(&f, &f, &g);
  }
  fe12 r;
  final_exp(&r, &f);
  return fe12_is_one(&r);
}
/* Signature::verify (sig_groupcheck = true, infinite pk rejected): 1 = valid */
int ref_verify(const uint8_t *sig192, const uint8_t *msg, size_t len, const uint8_t *pk96) {
  ensure_init();
  p1a pk;
  p2a sig;
  memcpy(&pk, pk96, 96);
  memcpy(&sig, sig192, 192);
  if (p1a_is_inf(&pk)) return 0;
  if (!p2a_is_inf(&sig) && !(p2_on_curve(&sig) && p2_in_group(&sig))) return 0;
  p2a H;
  hash_to_g2(&H, msg, len, DST_POP, 43);
  fe12 f, g;
  miller_loop_n(&f, &pk, &H, 1);
  if (!p2a_is_inf(&sig)) {
    p1a ng1 = G1;
    fe_neg(&ng1.y, &ng1.y);
    miller_loop_n(&g, &ng1, &sig, 1);
    fe12_mul(&f, &f, &g);
  }
  fe12 r;
  final_exp(&r, &f);
  return fe12_is_one(&r);
}
void ref_hash_to_g2(const uint8_t *msg, size_t len, const uint8_t *dst, size_t dlen, uint8_t *out192) {
  ensure_init();
  p2a H;
  hash_to_g2(&H, msg, len, dst, dlen);
  memcpy(out192, &H, 192);
}
static void sk_words(u64 *k, const uint8_t *sk32) {
  for (int i = 0; i < 4; i++) {
    k[i] = 0;
    for (int b = 0; b < 8; b++) k[i] |= (u64)sk32[31 - 8 * i - b] << (8 * b);
  }
}
void ref_sk_to_pk(const uint8_t *sk32, uint8_t *out96) {
  ensure_init();
  u64 k[4];
  sk_words(k, sk32);
  p1j g, r;
  p1_from_aff(&g, &G1);
  p1_mul_words(&r, &g, k, 256);
  p1a a;
  p1_to_aff(&a, &r);
  memcpy(out96, &a, 96);
}
void ref_sign(const uint8_t *sk32, const uint8_t *msg, size_t len, uint8_t *out192) {
  ensure_init();
  u64 k[4];
  sk_words(k, sk32);
  p2a H;
  hash_to_g2(&H, msg, len, DST_POP, 43);
  p2j h, r;
  p2_from_aff(&h, &H);
  p2_mul_words(&r, &h, k, 256);
  p2a a;
  p2_to_aff(&a, &r);
  memcpy(out192, &a, 192);
}
/* ZCash compressed G2 encoding (for byte-level parity checks) */
void ref_g2_compress(const uint8_t *in192, uint8_t *out96) {
  ensure_init();
  p2a a;
  memcpy(&a, in192, 192);
  memset(out96, 0, 96);
  if (p2a_is_inf(&a)) { out96[0] = 0xc0; return; }
  fe x1, x0;
  fe_to_plain(&x1, &a.x.b);
  fe_to_plain(&x0, &a.x.a);
  for (int i = 0; i < 48; i++) {
    out96[47 - i] = (uint8_t)(x1.v[i / 8] >> (8 * (i % 8)));
    out96[95 - i] = (uint8_t)(x0.v[i / 8] >> (8 * (i % 8)));
  }
  out96[0] |= 0x80 | (fe2_lex_largest(&a.y) ? 0x20 : 0);
}
