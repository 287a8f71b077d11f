// Test-only host build of the engine's __host__ __device__ arithmetic
// (grandine_amd/csrc/*.h), so the container without a GPU can check the exact code
// the gfx950 kernels run against the Python oracle.  Not part of the product: the
// shipped library (libgrandine_bls.so) has no CPU path.
#include <cstring>
#include <vector>

#include "../../grandine_amd/csrc/bls_hash.h"
#include "../../grandine_amd/csrc/bls_pairing.h"
#include "../../grandine_amd/csrc/bls_wave12.h"
#include "../../grandine_amd/csrc/bls_field28.h"
#include "../../grandine_amd/csrc/bls_curve28.h"
#include "../../grandine_amd/csrc/bls_inv.h"

using namespace gbls;

static const uint8_t POP[] = "BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_";

extern "C" {

void h_fp_mul(const uint32_t *a, const uint32_t *b, uint32_t *r) {
  fp x, y, z;
  std::memcpy(x.l, a, 48);
  std::memcpy(y.l, b, 48);
  fp_mul(z, x, y);
  std::memcpy(r, z.l, 48);
}

// radix-2^28 layer (bls_field28.h) through the engine form: op 0 = round trip of a,
// 1 = a b, 2 = a b + c d (mul2), 3 = a - b (sub, then mul by 1 path), 4 = Fp2 (a + b u)(c + d u)
// into r (and r2), 5 = Fp2 square of a + b u, 6 = is_zero(a - b)
int h_r28_op(int op, const uint32_t *a, const uint32_t *b, const uint32_t *c, const uint32_t *d,
             uint32_t *r, uint32_t *r2) {
  fp x[4];
  std::memcpy(x[0].l, a, 48);
  std::memcpy(x[1].l, b, 48);
  std::memcpy(x[2].l, c, 48);
  std::memcpy(x[3].l, d, 48);
  r28::fe e[4];
  for (int i = 0; i < 4; i++) r28::from_fp(e[i], x[i]);
  r28::fe o;
  r28::fe2 o2;
  fp z, z2;
  int ret = 0;
  switch (op) {
    case 0: o = e[0]; break;
    case 1: r28::mul(o, e[0], e[1]); break;
    case 2: r28::mul2(o, e[0], e[1], e[2], e[3]); break;
    case 3: r28::sub(o, e[0], e[1]); break;
    case 4:
    case 5: {
      r28::fe2 u = {e[0], e[1]}, v = {e[2], e[3]};
      if (op == 4)
        r28::fe2_mul(o2, u, v);
      else
        r28::fe2_sqr(o2, u);
      o = o2.c0;
      r28::to_fp(z2, o2.c1);
      std::memcpy(r2, z2.l, 48);
      break;
    }
    case 6: r28::sub(o, e[0], e[1]); ret = r28::is_zero(o); break;
    default: return -1;
  }
  r28::to_fp(z, o);
  std::memcpy(r, z.l, 48);
  return ret;
}

// radix-2^28 sparse Miller products (bls_field28.h) against the engine's (bls_pairing.h) on
// random operands: sp x sp, then a chain of dense x sparse products; and the uniform scalar
// of sp_from_engine.  Returns the number of mismatching Fp coefficients.
static uint64_t h_rng = 1;
static void h_rand_fp(fp &a) {
  for (int i = 0; i < 12; i++) {
    h_rng = h_rng * 6364136223846793005ull + 1442695040888963407ull;
    a.l[i] = (uint32_t)(h_rng >> 32);
  }
  a.l[11] &= 0x0fffffff;  // < 2^380 < p
}
static void h_rand_fp2(fp2 &a) {
  h_rand_fp(a.c0);
  h_rand_fp(a.c1);
}
static int h_fp_differs(const fp &x, const fp &y) {
  fp d;
  fp_sub(d, x, y);
  return !fp_is_zero(d);
}
static void h_to28(r28::fe2 &r, const fp2 &a) {
  r28::from_fp(r.c0, a.c0);
  r28::from_fp(r.c1, a.c1);
}
static int h_cmp12(const fp12 &e, const r28::fe12 &q) {
  const fp *ev[12] = {&e.c0.c0.c0, &e.c0.c0.c1, &e.c0.c1.c0, &e.c0.c1.c1, &e.c0.c2.c0, &e.c0.c2.c1,
                      &e.c1.c0.c0, &e.c1.c0.c1, &e.c1.c1.c0, &e.c1.c1.c1, &e.c1.c2.c0, &e.c1.c2.c1};
  const r28::fe *qv[12] = {&q.c0.c0.c0, &q.c0.c0.c1, &q.c0.c1.c0, &q.c0.c1.c1, &q.c0.c2.c0,
                           &q.c0.c2.c1, &q.c1.c0.c0, &q.c1.c0.c1, &q.c1.c1.c0, &q.c1.c1.c1,
                           &q.c1.c2.c0, &q.c1.c2.c1};
  int bad = 0;
  for (int i = 0; i < 12; i++) {
    fp t;
    r28::to_fp(t, *qv[i]);
    bad += h_fp_differs(t, *ev[i]);
  }
  return bad;
}
int h_r28_tower_check(uint64_t seed, int rounds, int chain) {
  h_rng = seed;
  int bad = 0;
  for (int it = 0; it < rounds; it++) {
    sp034 ea, eb;
    r28::sp qa, qb;
    h_rand_fp2(ea.a0), h_rand_fp2(ea.a2), h_rand_fp2(ea.a3);
    h_rand_fp2(eb.a0), h_rand_fp2(eb.a2), h_rand_fp2(eb.a3);
    h_to28(qa.a0, ea.a0), h_to28(qa.a2, ea.a2), h_to28(qa.a3, ea.a3);
    h_to28(qb.a0, eb.a0), h_to28(qb.a2, eb.a2), h_to28(qb.a3, eb.a3);
    fp12 ef;
    r28::fe12 qf;
    sp_mul_sp(ef, ea, eb);
    r28::sp_mul_sp(qf, qa, qb);
    bad += h_cmp12(ef, qf);
    {  // the lazy sparse x sparse product (one reduction per output coordinate)
      r28::fe12 ql;
      r28::sp_mul_sp_lazy(ql, qa, qb);
      bad += h_cmp12(ef, ql);
    }
    for (int j = 0; j < chain; j++) {
      h_rand_fp2(ea.a0), h_rand_fp2(ea.a2), h_rand_fp2(ea.a3);
      h_to28(qa.a0, ea.a0), h_to28(qa.a2, ea.a2), h_to28(qa.a3, ea.a3);
      fp12_mul_034(ef, ef, ea);
      uint32_t st[154 * 3];
      switch (j & 3) {  // every form, chained (each one's outputs are the next one's inputs)
        case 0: r28::fe12_mul_034(qf, qf, qa); break;
        case 1: r28::fe12_mul_034_st(qf, qf, qa, st + 1, 3); break;
        case 2: r28::fe12_mul_034_lazy(qf, qa); break;
        default: r28::fe12_mul_034_lazy_st(qf, qa, st + 2, 3); break;
      }
    }
    bad += h_cmp12(ef, qf);
    // sp_from_engine: engine line at (x, y, c) up to one scalar for all six coefficients
    fp2 L0, L2, L3;
    g1s P;
    h_rand_fp2(L0), h_rand_fp2(L2), h_rand_fp2(L3);
    h_rand_fp(P.x), h_rand_fp(P.y), h_rand_fp(P.c);
    sp034 es;
    line_eval_s(es, L0, L2, L3, P);
    r28::sp qs;
    r28::sp_from_engine(qs, L0, L2, L3, P.x, P.y, P.c);
    const fp *ev[6] = {&es.a0.c0, &es.a0.c1, &es.a2.c0, &es.a2.c1, &es.a3.c0, &es.a3.c1};
    const r28::fe *qv[6] = {&qs.a0.c0, &qs.a0.c1, &qs.a2.c0, &qs.a2.c1, &qs.a3.c0, &qs.a3.c1};
    fp q0;
    r28::to_fp(q0, *qv[0]);
    for (int i = 1; i < 6; i++) {  // q_i e_0 == q_0 e_i
      fp qi, l, r;
      r28::to_fp(qi, *qv[i]);
      fp_mul(l, qi, *ev[0]);
      fp_mul(r, q0, *ev[i]);
      bad += h_fp_differs(l, r);
    }
  }
  return bad;
}

// the radix-2^28 Miller line steps (bls_curve28.h line_dbl28 / line_add28, k_lines_lane28)
// against the engine's (bls_pairing.h line_dbl / line_add_aff) over the 68 events from a
// random Q: every line coefficient and the final T equal as field elements
int h_r28_lines_check(uint64_t seed) {
  h_rng = seed;
  g2a Q;
  h_rand_fp2(Q.x), h_rand_fp2(Q.y);
  g2h T;
  T.x = Q.x, T.y = Q.y;
  fp2_one(T.z);
  r28::g2h28 T28;
  r28::fe2 qx, qy;
  h_to28(qx, Q.x), h_to28(qy, Q.y);
  T28.x = qx, T28.y = qy;
  r28::f_one(T28.z);
  int bad = 0;
  for (int e = 0; e < ML_EVENTS; e++) {
    fp2 L[6], E[3];
    auto put = [&](int c, const r28::fe2 &v) {
      r28::to_fp(L[c].c0, v.c0);
      r28::to_fp(L[c].c1, v.c1);
    };
    if (ev_is_dbl(e)) {
      line_dbl(T, E[0], E[1], E[2]);
      r28::line_dbl28(T28, put);
    } else {
      line_add_aff(T, Q, E[0], E[1], E[2]);
      r28::line_add28(T28, qx, qy, put);
    }
    for (int k = 0; k < 3; k++)
      bad += h_fp_differs(L[2 * k].c0, E[k].c0) + h_fp_differs(L[2 * k].c1, E[k].c1);
    // the stored form: repacked radix-2^28 words read back (load12) are the same value
    fp w;
    r28::fe back;
    r28::store12(w, T28.x.c0);
    r28::load12(back, w);
    fp a, b;
    r28::to_fp(a, back);
    r28::to_fp(b, T28.x.c0);
    bad += h_fp_differs(a, b);
  }
  const fp2 *ev[3] = {&T.x, &T.y, &T.z};
  const r28::fe2 *qv[3] = {&T28.x, &T28.y, &T28.z};
  for (int k = 0; k < 3; k++) {
    fp t0, t1;
    r28::to_fp(t0, qv[k]->c0);
    r28::to_fp(t1, qv[k]->c1);
    bad += h_fp_differs(t0, ev[k]->c0) + h_fp_differs(t1, ev[k]->c1);
  }
  return bad;
}

int h_g1_decompress(const uint8_t *in, int validate, uint8_t *out96) {
  g1a a;
  int s = g1_decompress(a, in);
  if (s == ST_SUCCESS && validate) {
    if (aff_is_inf(a))
      s = ST_PK_IS_INFINITY;
    else if (!g1_in_group(a))
      s = ST_NOT_IN_GROUP;
  }
  std::memcpy(out96, &a, 96);
  return s;
}
int h_g2_decompress(const uint8_t *in, uint8_t *out192) {
  g2a a;
  int s = g2_decompress(a, in);
  std::memcpy(out192, &a, 192);
  return s;
}
int h_g2_in_group(const uint8_t *in192) {
  g2a a;
  std::memcpy(&a, in192, 192);
  return g2_in_group(a);
}
void h_g1_compress(const uint8_t *in96, uint8_t *out48) {
  g1a a;
  std::memcpy(&a, in96, 96);
  g1_compress(out48, a);
}
void h_g2_compress(const uint8_t *in192, uint8_t *out96) {
  g2a a;
  std::memcpy(&a, in192, 192);
  g2_compress(out96, a);
}
void h_hash_to_g2(const uint8_t *msg, uint32_t len, const uint8_t *dst, uint32_t dlen,
                  uint8_t *out192) {
  g2j h;
  hash_to_g2(h, msg, len, dst_ref{dst, dlen});
  g2a a;
  jac_to_aff(a, h);
  std::memcpy(out192, &a, 192);
}
// G1 aggregate of n affine points (same code path as k_g1_aggregate_seg, one lane)
int h_g1_aggregate(const uint8_t *pks96, uint32_t n, uint8_t *out96) {
  g1j acc;
  jac_set_inf(acc);
  for (uint32_t i = 0; i < n; i++) {
    g1a p;
    std::memcpy(&p, pks96 + 96 * i, 96);
    jac_add_aff(acc, acc, p);
  }
  g1a r;
  jac_to_aff(r, acc);
  std::memcpy(out96, &r, 96);
  return n ? ST_SUCCESS : ST_AGGR_TYPE_MISMATCH;
}
// windowed G1 scalar product (k_mv_g1mul_lane) against double-and-add: 1 if equal
int h_g1_mul_w3_check(const uint8_t *pk96, uint64_t k) {
  g1a p;
  std::memcpy(&p, pk96, 96);
  g1j a, b;
  g1_mul_u64_w3(a, p, k);
  mul_u64(b, p, k);
  return jac_eq(a, b);
}
void h_sk_to_pk(const uint8_t *sk32, uint8_t *out96) {
  uint32_t s[8];
  for (int i = 0; i < 8; i++) {
    const uint8_t *q = sk32 + 4 * (7 - i);
    s[i] = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | q[3];
  }
  g1a g;
  fp_set(g.x, k::G1X_M);
  fp_set(g.y, k::G1Y_M);
  g1j acc;
  jac_set_inf(acc);
  for (int i = 255; i >= 0; i--) {
    jac_dbl(acc, acc);
    if ((s[i >> 5] >> (i & 31)) & 1) jac_add_aff(acc, acc, g);
  }
  g1a a;
  jac_to_aff(a, acc);
  std::memcpy(out96, &a, 96);
}
// stage-by-stage hash_to_G2 intermediates (layout of tools/debug/h2c_dbg.hip's Out)
struct H2cStages {
  fp2 u[2];
  g2j q[2];
  g2j sum;
  g2j h;
  g2a ha;
  fp sq_n, sq_gamma, inv_in, inv_out;
};
void h_h2c_stages(const uint8_t *msg, uint32_t len, const uint8_t *dst, uint32_t dlen, uint8_t *out) {
  H2cStages o;
  std::memset(&o, 0, sizeof o);
  hash_to_field_g2(o.u, msg, len, dst_ref{dst, dlen});
  map_to_g2(o.q[0], o.u[0]);
  map_to_g2(o.q[1], o.u[1]);
  g2j a = o.q[0];
  jac_add(a, a, o.q[1]);
  o.sum = a;
  clear_cofactor_g2(o.h, a);
  jac_to_aff(o.ha, o.h);
  o.inv_in = o.u[0].c0;
  fp_inv(o.inv_out, o.inv_in);
  fp_pow_pm3d4(o.sq_gamma, o.u[0].c1);
  std::memcpy(out, &o, sizeof o);
}
uint32_t h_h2c_stages_size() { return sizeof(H2cStages); }

// ---- host emulation of the wave-cooperative Fp12 engine (bls_wave12.h): every round
// runs lanes 0..63 in order, exactly as the single-wave device workgroup does.
static void w12_mul_host(uint32_t *c, const uint32_t *a, const uint32_t *b) {
  static uint32_t ws[W12_WS_WORDS];
  static w12_plan pl[64];
  static bool init = false;
  if (!init) {
    for (int l = 0; l < 64; l++) {
      w12_plan_load(pl[l], l);
      w12_r_ws_init(l, ws);
    }
    init = true;
  }
  for (int l = 0; l < 64; l++) w12_r_mul(l, pl[l], a, b, ws);
  for (int l = 0; l < 64; l++) w12_r_post1(l, pl[l], ws);
  for (int l = 0; l < 64; l++) w12_r_post2(l, pl[l], ws);
  for (int l = 0; l < 64; l++) w12_r_post3(l, pl[l], ws, c);
}
static void w12_conj_host(uint32_t *c, const uint32_t *a) {
  for (int l = 0; l < 64; l++) w12_r_conj(l, a, c);
}
static void w12_exp_x_host(uint32_t *c, const uint32_t *a) {
  for (int l = 0; l < 64; l++) w12_r_copy(l, a, c);
  for (int i = 62; i >= 0; i--) {
    w12_mul_host(c, c, c);
    if ((k::X_ABS >> i) & 1) w12_mul_host(c, c, a);
  }
  w12_conj_host(c, c);
}
// k_final_verdict's inversion-free chain on the host engine emulation
static bool w12_final_verdict_host(const fp12 &f0) {
  uint32_t f[144], G[144], A[144], B[144], T[144], X[144];
  std::memcpy(f, &f0, sizeof f);
  if (w12_is_zero_image(f)) return false;
  for (int l = 0; l < 64; l++) w12_r_frob2(l, f, G);
  w12_mul_host(G, G, f);
  w12_exp_x_host(A, G);
  w12_conj_host(X, G);
  w12_mul_host(A, A, X);
  w12_exp_x_host(B, A);
  w12_conj_host(X, A);
  w12_mul_host(A, B, X);
  w12_exp_x_host(B, A);
  for (int l = 0; l < 64; l++) w12_r_frob(l, A, X);
  w12_mul_host(B, B, X);
  w12_exp_x_host(T, B);
  w12_exp_x_host(A, T);
  for (int l = 0; l < 64; l++) w12_r_frob2(l, B, X);
  w12_mul_host(A, A, X);
  w12_conj_host(X, B);
  w12_mul_host(A, A, X);
  w12_mul_host(X, G, G);
  w12_mul_host(X, X, G);
  w12_mul_host(A, A, X);
  return w12_is_fp6_image(A);
}
// the device verdict and the textbook final exponentiation (bls_pairing.h) on one value
int h_w12_verdict(const uint8_t *f576) {
  fp12 f;
  std::memcpy(&f, f576, 576);
  return w12_final_verdict_host(f);
}
int h_final_exp_is_one(const uint8_t *f576) {
  fp12 f, r;
  std::memcpy(&f, f576, 576);
  final_exp(r, f);
  return fp12_is_one(r);
}
// Miller partial of a multi_verify batch on the host (the device pipeline's formulas)
void h_fp12_mul(const uint8_t *a576, const uint8_t *b576, uint8_t *out576) {
  fp12 a, b, r;
  std::memcpy(&a, a576, 576);
  std::memcpy(&b, b576, 576);
  fp12_mul(r, a, b);
  std::memcpy(out576, &r, 576);
}

void h_fp12_mul_w12(const uint8_t *a576, const uint8_t *b576, uint8_t *out576) {
  uint32_t a[144], b[144], c[144];
  std::memcpy(a, a576, 576);
  std::memcpy(b, b576, 576);
  w12_mul_host(c, a, b);
  std::memcpy(out576, c, 576);
}
void h_fp12_mul_ref(const uint8_t *a576, const uint8_t *b576, uint8_t *out576) {
  fp12 a, b, c;
  std::memcpy(&a, a576, 576);
  std::memcpy(&b, b576, 576);
  fp12_mul(c, a, b);
  std::memcpy(out576, &c, 576);
}
// bls_inv.h: the safegcd inversion of the final exponentiation's easy part
void h_fp_inv_var(const uint8_t *a48, uint8_t *out48) {
  fp a, r;
  std::memcpy(a.l, a48, 48);
  fp_inv_var(r, a);
  std::memcpy(out48, r.l, 48);
}
int h_fp_inv_check(const uint8_t *a48, uint8_t *out48) {
  fp a, r, t;
  std::memcpy(a.l, a48, 48);
  fp_inv(r, a);
  std::memcpy(out48, r.l, 48);
  fp_mul(t, r, a);
  return fp_is_one(t);
}

// Sequential emulation of the device pipeline (gbls_capi.hip pipeline_partials +
// pipeline_final): same per-lane functions, the Miller product over all pairs of a
// segment formed event by event (as the device tree + Horner do), and the final
// exponentiation on the emulated wave engine.
static void pipeline(const uint8_t *msgs, const uint32_t *msg_off, const uint8_t *sigs192,
                     const uint8_t *pks96, const uint64_t *rands, const int32_t *pre, uint32_t n,
                     const uint32_t *seg_off, uint32_t nseg, int32_t *verdicts) {
  for (uint32_t s = 0; s < nseg; s++) {
    uint32_t b = seg_off[s], e_ = seg_off[s + 1];
    uint32_t np = e_ - b + 1;
    std::vector<uint32_t> L((size_t)np * ML_EVENTS * 72);
    std::vector<g1s> P(np);
    g2j S;
    jac_set_inf(S);
    int err = e_ == b;
    for (uint32_t i = b; i < e_; i++) {
      const uint8_t *m = msg_off ? msgs + msg_off[i] : msgs + 32 * i;
      uint32_t len = msg_off ? msg_off[i + 1] - msg_off[i] : 32;
      fp2 u[2];
      hash_to_field_g2(u, m, len, dst_ref{POP, 43});  // k_h2c_field
      g2j q0, q1, h;
      map_to_g2(q0, u[0]);                            // k_h2c_map
      map_to_g2(q1, u[1]);
      jac_add(q0, q0, q1);                            // k_h2c_clear
      clear_cofactor_g2(h, q0);
      g2a H;
      jac_to_aff(H, h);
      g1a pk;
      g2a sig;
      std::memcpy(&pk, pks96 + 96 * i, 96);
      std::memcpy(&sig, sigs192 + 192 * i, 192);
      uint64_t r = rands ? rands[i] : 1;
      g1j t;                                          // k_mv_g1mul (no inversion)
      mul_u64(t, pk, r);
      g1s_from_jac(P[i - b], t);
      err |= aff_is_inf(pk) || (pre && pre[i]);
      g2j R;                                          // k_mv_g2mul
      mul_u64(R, sig, r);
      jac_add(S, S, R);                               // k_seg_g2_sum
      lines_of(L.data(), np, i - b, H);               // k_lines
    }
    fp_set(P[np - 1].x, k::G1X_M);
    fp_set(P[np - 1].y, k::G1NEGY_M);
    fp_one(P[np - 1].c);
    g2a Sa;
    jac_to_aff(Sa, S);
    lines_of(L.data(), np, np - 1, Sa);
    // k_ml_leaf / k_ml_reduce / k_ml_horner
    fp12 f;
    for (int e = 0; e < ML_EVENTS; e++) {
      fp12 M;
      fp12_one(M);
      for (uint32_t j = 0; j < np; j++) {
        fp2 L0, L2, L3;
        sp034 sp;
        line_get(L.data(), np, j, e, L0, L2, L3);
        line_eval_s(sp, L0, L2, L3, P[j]);
        fp12_mul_034(M, M, sp);
      }
      if (e == 0) {
        f = M;
      } else {
        if (ev_is_dbl(e)) fp12_sqr(f, f);
        fp12_mul(f, f, M);
      }
    }
    fp12_conj(f, f);
    verdicts[s] = (!err && w12_final_verdict_host(f)) ? ST_SUCCESS : ST_VERIFY_FAIL;
  }
}

// gbls_verify: sig subgroup check + single-set segment with r = 1
int h_verify(const uint8_t *sig192, const uint8_t *msg, uint32_t len, const uint8_t *pk96) {
  g2a sig;
  std::memcpy(&sig, sig192, 192);
  int32_t pre = !(aff_is_inf(sig) || (g2_on_curve(sig) && g2_in_group(sig)));
  uint32_t moff[2] = {0, len}, soff[2] = {0, 1};
  int32_t v;
  pipeline(msg, moff, sig192, pk96, nullptr, &pre, 1, soff, 1, &v);
  return v;
}
int h_multi_verify(const uint8_t *msgs32, const uint8_t *sigs192, const uint8_t *pks96,
                   const uint64_t *rands, uint32_t n) {
  uint32_t soff[2] = {0, n};
  int32_t v;
  pipeline(msgs32, nullptr, sigs192, pks96, rands, nullptr, n, soff, 1, &v);
  return v;
}

// the lane-regime cofactor clearing in the radix-2^28 layer (bls_curve28.h) against the
// engine's (bls_hash.h clear_cofactor_g2) on Q0 + Q1 of a message: 1 when the points agree
int h_r28_clear_check(const uint8_t *msg, uint32_t len) {
  fp2 u[2];
  hash_to_field_g2(u, msg, len, dst_ref{POP, 43});
  g2j q0, q1, want, got;
  map_to_g2(q0, u[0]);
  map_to_g2(q1, u[1]);
  jac_add(q0, q0, q1);
  clear_cofactor_g2(want, q0);
  r28::g2j28 a, h, hs;
  r28::g2j_in(a, q0);
  r28::clear_cofactor28(h, a);
  r28::g2j_out(got, h);
  g2j gs;  // the lane kernels' staged form (affine chain bases)
  r28::clear_cofactor28_staged(hs, a);
  r28::g2j_out(gs, hs);
  return jac_eq(got, want) && jac_eq(gs, want) ? 1 : 0;
}

// G2 membership in radix 2^28 (bls_curve28.h g2_in_group28) against the engine's g2_in_group
// for a message's cleared hash point (in G2) and its uncleared map output (on E2, not in G2):
// 1 = both agree with the engine and the engine says (in, out)
int h_r28_g2check(const uint8_t *msg, uint32_t len) {
  fp2 u[2];
  hash_to_field_g2(u, msg, len, dst_ref{POP, 43});
  g2j q0, h;
  map_to_g2(q0, u[0]);
  clear_cofactor_g2(h, q0);
  int ok = 1;
  for (int k = 0; k < 2; k++) {
    g2a a;
    jac_to_aff(a, k == 0 ? h : q0);
    r28::g2a28 b;
    r28::from_fp(b.x.c0, a.x.c0), r28::from_fp(b.x.c1, a.x.c1);
    r28::from_fp(b.y.c0, a.y.c0), r28::from_fp(b.y.c1, a.y.c1);
    const bool want = g2_in_group(a), got = r28::g2_in_group28(b);
    ok &= (got == want) && (want == (k == 0));
  }
  return ok;
}

// G1 [k]P in radix 2^28 (bls_curve28.h g1_mul_u64_w3_28 + g1s_from_jac28) against the engine's
// g1_mul_u64_w3 + g1s_from_jac: the same point up to the scaled form's Fp factor (x / c, y / c
// compared through cross products), for n seeded (P, k); 0 = all equal
int h_r28_g1mul_check(uint64_t seed, int n) {
  int bad = 0;
  for (int t = 0; t < n; t++) {
    g1a base, gen;
    fp_set(gen.x, k::G1X_M);
    fp_set(gen.y, k::G1Y_M);
    {
      g1j g;
      g1_mul_u64_w3(g, gen, (seed + 977 * t) | 1);
      jac_to_aff(base, g);
    }
    const uint64_t k = (seed * 0x9E3779B97F4A7C15ull) ^ (0xD1B54A32D192ED03ull * (t + 1));
    g1j want;
    g1_mul_u64_w3(want, base, k);
    g1s ws, gs;
    g1s_from_jac(ws, want);
    r28::g1j28 got;
    r28::g1_mul_u64_w3_28(got, base, k);
    r28::g1s_from_jac28(gs, got);
    fp a, b;  // x_w c_g == x_g c_w, y_w c_g == y_g c_w  (c = Z^3, x = X Z)
    fp_mul(a, ws.x, gs.c);
    fp_mul(b, gs.x, ws.c);
    bool ok = fp_eq(a, b);
    fp_mul(a, ws.y, gs.c);
    fp_mul(b, gs.y, ws.c);
    ok = ok && fp_eq(a, b) && !fp_is_zero(gs.c);
    bad += !ok;
  }
  return bad;
}

}  // extern "C"

// The lazy doubling and additions (bls_curve28.h jac_dbl28 / jac_add28 / jac_add_aff28) against
// bls_curve.h's templates over the reduced f_ operations, from inputs at the top of its contract (coordinates raised by p:
// normalized, < 2.03 p; X and Y raised again every few steps), through n chained doublings of
// r28::fe2 and r28::fe points (the formula is algebraic: no curve point needed); with
// GBLS_R28_CHECK every combination's limb contract is checked too.  0 = all equal
static uint32_t h_rng32(uint64_t &s) {
  s = s * 6364136223846793005ull + 1442695040888963407ull;
  return (uint32_t)(s >> 32);
}
static void h_rand(r28::fe &r, uint64_t &s) {
  fp x;
  for (int i = 0; i < 12; i++) x.l[i] = h_rng32(s);
  x.l[11] &= 0x0fffffffu;  // < 2^380 < p
  r28::from_fp(r, x);
}
static void h_rand(r28::fe2 &r, uint64_t &s) {
  h_rand(r.c0, s);
  h_rand(r.c1, s);
}
static void h_raise(r28::fe &a) {
  constexpr r28::fe P = {{GBLS_R28_P}};
  r28::add_n(a, a, P);
}
static void h_raise(r28::fe2 &a) {
  h_raise(a.c0);
  h_raise(a.c1);
}
static bool h_same(const r28::fe &a, const r28::fe &b) {
  fp x, y;
  r28::to_fp(x, a);
  r28::to_fp(y, b);
  return fp_eq(x, y);
}
static bool h_same(const r28::fe2 &a, const r28::fe2 &b) { return h_same(a.c0, b.c0) && h_same(a.c1, b.c1); }
template <class F>
static int h_dbl_chain(uint64_t seed, int n) {
  uint64_t s = seed;
  jac<F> a, b;
  h_rand(a.x, s);
  h_rand(a.y, s);
  h_rand(a.z, s);
  b = a;
  h_raise(a.x);
  h_raise(a.y);
  h_raise(a.z);
  int bad = 0;
  for (int i = 0; i < n; i++) {
    r28::jac_dbl28(a, a);
    gbls::jac_dbl<F>(b, b);
    bad += !(h_same(a.x, b.x) && h_same(a.y, b.y) && h_same(a.z, b.z));
    if (i % 3 == 1) {  // + a Jacobian point (its lazy copy raised to < 2.03 p)
      jac<F> c, cr;
      h_rand(c.x, s);
      h_rand(c.y, s);
      h_rand(c.z, s);
      cr = c;
      h_raise(cr.x);
      h_raise(cr.z);
      r28::jac_add28(a, a, cr);
      gbls::jac_add<F>(b, b, c);
      bad += !(h_same(a.x, b.x) && h_same(a.y, b.y) && h_same(a.z, b.z));
    }
    if (i % 3 == 2) {  // + an affine point
      aff<F> q;
      h_rand(q.x, s);
      h_rand(q.y, s);
      r28::jac_add_aff28<true>(a, a, q);
      gbls::jac_add_aff<F>(b, b, q);
      bad += !(h_same(a.x, b.x) && h_same(a.y, b.y) && h_same(a.z, b.z));
    }
    if (i % 5 == 2) {
      h_raise(a.x);
      h_raise(a.y);
    }
  }
  return bad;
}
extern "C" {
int h_r28_dbl_check(uint64_t seed, int n) {
  return h_dbl_chain<r28::fe2>(seed, n) + h_dbl_chain<r28::fe>(seed ^ 0x5bd1e995u, n);
}

}  // extern "C"
