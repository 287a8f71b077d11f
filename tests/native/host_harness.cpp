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
// k_av_miller + k_final_verify for one set
int h_verify(const uint8_t *sig192, const uint8_t *msg, uint32_t len, const uint8_t *pk96) {
  g2a sig;
  g1a pk;
  std::memcpy(&sig, sig192, 192);
  std::memcpy(&pk, pk96, 96);
  if (aff_is_inf(pk)) return ST_VERIFY_FAIL;
  if (!aff_is_inf(sig) && !g2_in_group(sig)) return ST_VERIFY_FAIL;
  g2j h;
  hash_to_g2(h, msg, len, dst_ref{POP, 43});
  g2a ha;
  jac_to_aff(ha, h);
  fp12 f, t;
  miller_loop(f, pk, ha);
  if (!aff_is_inf(sig)) {
    g1a ng1;
    fp_set(ng1.x, k::G1X_M);
    fp_set(ng1.y, k::G1NEGY_M);
    miller_loop(t, ng1, sig);
    fp12_mul(f, f, t);
  }
  fp12 r;
  final_exp(r, f);
  return fp12_is_one(r) ? ST_SUCCESS : ST_VERIFY_FAIL;
}
// the multi_verify stage sequence (k_hash_to_g2, k_mv_g1mul, k_mv_g2mul, k_seg_g2_sum,
// k_miller, k_seg_fp12_prod, k_seg_partial, k_final_verify) for one segment
int h_multi_verify(const uint8_t *msgs32, const uint8_t *sigs192, const uint8_t *pks96,
                   const uint64_t *rands, uint32_t n) {
  fp12 F;
  fp12_one(F);
  g2j S;
  jac_set_inf(S);
  int bad = n == 0;
  for (uint32_t i = 0; i < n; i++) {
    g2a sig, H;
    g1a pk, P;
    std::memcpy(&sig, sigs192 + 192 * i, 192);
    std::memcpy(&pk, pks96 + 96 * i, 96);
    g2j h;
    hash_to_g2(h, msgs32 + 32 * i, 32, dst_ref{POP, 43});
    jac_to_aff(H, h);
    g1j t;
    mul_u64(t, pk, rands[i]);
    jac_to_aff(P, t);
    bad |= aff_is_inf(pk);
    g2j R;
    mul_u64(R, sig, rands[i]);
    jac_add(S, S, R);
    fp12 f;
    miller_loop(f, P, H);
    fp12_mul(F, F, f);
  }
  g2a sa;
  jac_to_aff(sa, S);
  g1a ng1;
  fp_set(ng1.x, k::G1X_M);
  fp_set(ng1.y, k::G1NEGY_M);
  fp12 m;
  miller_loop(m, ng1, sa);
  fp12_mul(F, F, m);
  fp12 r;
  final_exp(r, F);
  return (!bad && fp12_is_one(r)) ? ST_SUCCESS : ST_VERIFY_FAIL;
}

}  // extern "C"
