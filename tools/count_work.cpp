// Freezes the algorithmic work W of every pipeline stage: the
// engine's own __host__ __device__ formulas (grandine_amd/csrc/*.h) compiled for the host
// with -DGBLS_COUNT_FPMUL, which counts every 12-limb Montgomery product (fp_mul; a
// squaring is a product).  Serial (lane-per-item) formula counts are the unit of work:
// the device's quad gangs and wave-cooperative Fp12 engine spread the same products over
// more lanes, and inversions by binary GCD count only their final Montgomery product.
//
// Build + run:  g++ -O2 -std=c++17 -DGBLS_COUNT_FPMUL -D__HIP_PLATFORM_AMD__ \
//   -I/opt/rocm/include tools/count_work.cpp -o /tmp/count_work && /tmp/count_work
#include <cstdio>
#include <cstring>
#include <random>

#include "../grandine_amd/csrc/bls_hash.h"
#include "../grandine_amd/csrc/bls_pairing.h"

using namespace gbls;

thread_local unsigned long long gbls::g_fpmul_count = 0;

static unsigned long long tick() {
  unsigned long long c = g_fpmul_count;
  g_fpmul_count = 0;
  return c;
}

int main() {
  const int NS = 64;  // averaged over seeded inputs (scalar popcounts vary)
  std::mt19937_64 rng(20251016);
  static const uint8_t POP[] = "BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_";
  double w_map = 0, w_clear = 0, w_g1mul = 0, w_g2mul = 0, w_g2add = 0, w_lines = 0, w_eval = 0,
         w_spsp = 0, w_fexp = 0, w_fp12mul = 0, w_fp12sqr = 0, w_g1madd = 0, w_g2check = 0;
  g1a G1;
  fp_set(G1.x, k::G1X_M);
  fp_set(G1.y, k::G1Y_M);
  for (int s = 0; s < NS; s++) {
    uint8_t msg[32];
    for (int i = 0; i < 32; i++) msg[i] = (uint8_t)rng();
    fp2 u[2];
    hash_to_field_g2(u, msg, 32, dst_ref{POP, 43});
    tick();
    g2j q0, q1;
    map_to_g2(q0, u[0]);
    map_to_g2(q1, u[1]);
    w_map += tick();
    jac_add(q0, q0, q1);
    g2j h;
    clear_cofactor_g2(h, q0);
    g2a H;
    jac_to_aff(H, h);
    w_clear += tick();
    uint64_t r = rng() | 1;
    // a G1 point: r' * G1 affine
    g1j t;
    mul_u64(t, G1, rng() | 1);
    g1a pk;
    jac_to_aff(pk, t);
    tick();
    mul_u64(t, pk, r);
    g1a P;
    jac_to_aff(P, t);
    w_g1mul += tick();
    g2j R;
    mul_u64(R, H, r);
    w_g2mul += tick();
    g2j acc;
    jac_from_aff(acc, H);
    jac_add(acc, acc, R);
    w_g2add += tick();
    static uint32_t L[ML_EVENTS * 72];
    lines_of(L, 1, 0, H);
    w_lines += tick();
    fp2 L0, L2, L3;
    sp034 sa, sb;
    line_get(L, 1, 0, 0, L0, L2, L3);
    line_eval(sa, L0, L2, L3, P);
    w_eval += tick();
    line_eval(sb, L0, L2, L3, P);
    tick();
    fp12 f;
    sp_mul_sp(f, sa, sb);
    w_spsp += tick();
    fp12 g2 = f;
    fp12_mul(g2, g2, f);
    w_fp12mul += tick();
    fp12_sqr(g2, g2);
    w_fp12sqr += tick();
    fp12 e;
    final_exp(e, g2);
    w_fexp += tick();
    g1j a1;
    jac_from_aff(a1, pk);
    jac_add_aff(a1, a1, P);
    w_g1madd += tick();
    (void)g2_in_group(H);
    w_g2check += tick();
  }
  const double n = NS;
  std::printf("{\"fp_products_per_unit\": {\n");
  std::printf("  \"map_to_g2_x2\": %.1f,\n", w_map / n);
  std::printf("  \"q0_plus_q1_clear_cofactor_to_affine\": %.1f,\n", w_clear / n);
  std::printf("  \"g1_mul_u64_to_affine\": %.1f,\n", w_g1mul / n);
  std::printf("  \"g2_mul_u64\": %.1f,\n", w_g2mul / n);
  std::printf("  \"g2_jacobian_add\": %.1f,\n", w_g2add / n);
  std::printf("  \"lines_68_events\": %.1f,\n", w_lines / n);
  std::printf("  \"line_eval\": %.1f,\n", w_eval / n);
  std::printf("  \"sparse_x_sparse\": %.1f,\n", w_spsp / n);
  std::printf("  \"fp12_mul\": %.1f,\n", w_fp12mul / n);
  std::printf("  \"fp12_sqr\": %.1f,\n", w_fp12sqr / n);
  std::printf("  \"final_exp\": %.1f,\n", w_fexp / n);
  std::printf("  \"g1_mixed_add\": %.1f,\n", w_g1madd / n);
  std::printf("  \"g2_subgroup_check\": %.1f\n", w_g2check / n);
  std::printf("}}\n");
  return 0;
}
