// Test-only host build of the engine's __host__ __device__ arithmetic
// (grandine_amd/csrc/*.h), so the container without a GPU can check the exact code
// the gfx950 kernels run against the Python oracle.  Not part of the product: the
// shipped library (libgrandine_bls.so) has no CPU path.
#include <cstring>

#include "../../grandine_amd/csrc/bls_hash.h"
#include "../../grandine_amd/csrc/bls_pairing.h"

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
// Sequential emulation of the device pipeline (gbls_capi.hip pipeline_partials +
// pipeline_final), stage by stage with the same per-lane functions as the kernels.
static void pipeline(const uint8_t *msgs, const uint32_t *msg_off, const uint8_t *sigs192,
                     const uint8_t *pks96, const uint64_t *rands, const int32_t *pre, uint32_t n,
                     const uint32_t *seg_off, uint32_t nseg, int32_t *verdicts) {
  for (uint32_t s = 0; s < nseg; s++) {
    fp12 acc;
    fp12_one(acc);
    g2j S;
    jac_set_inf(S);
    int err = seg_off[s + 1] == seg_off[s];
    for (uint32_t i = seg_off[s]; i < seg_off[s + 1]; i++) {
      const uint8_t *m = msg_off ? msgs + msg_off[i] : msgs + 32 * i;
      uint32_t len = msg_off ? msg_off[i + 1] - msg_off[i] : 32;
      fp2 u[2];
      hash_to_field_g2(u, m, len, dst_ref{POP, 43});                       // k_h2c_field
      g2j q0, q1, h;
      map_to_g2(q0, u[0]);                                                // k_h2c_map
      map_to_g2(q1, u[1]);
      jac_add(q0, q0, q1);                                                // k_h2c_clear
      clear_cofactor_g2(h, q0);
      g2h H;
      g2h_from_jac(H, h);
      g1a pk;
      g2a sig;
      std::memcpy(&pk, pks96 + 96 * i, 96);
      std::memcpy(&sig, sigs192 + 192 * i, 192);
      uint64_t r = rands ? rands[i] : 1;
      g1j t;                                                              // k_mv_g1mul
      mul_u64(t, pk, r);
      g1p P;
      g1p_from_jac(P, t);
      err |= aff_is_inf(pk) || (pre && pre[i]);
      g2j R;                                                              // k_mv_g2mul
      mul_u64(R, sig, r);
      jac_add(S, S, R);                                                   // k_seg_g2_sum
      fp12 f;
      miller_loop(f, P, H);                                               // k_miller
      fp12_mul(acc, acc, f);                                              // k_seg_fp12_prod
    }
    g1a ng1;
    fp_set(ng1.x, k::G1X_M);
    fp_set(ng1.y, k::G1NEGY_M);
    g1p PP;
    g1p_from_aff(PP, ng1);
    g2h QQ;
    g2h_from_jac(QQ, S);
    fp12 f;
    miller_loop(f, PP, QQ);
    fp12_mul(acc, acc, f);
    fp12 r;
    final_exp(r, acc);                                                    // k_fe_*
    verdicts[s] = (!err && fp12_is_one(r)) ? ST_SUCCESS : ST_VERIFY_FAIL;
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

}  // extern "C"
