// G2 in the radix-2^28 field layer (bls_field28.h) for the lane-regime cofactor clearing
// (DESIGN.md section 8's migration order): the engine's Jacobian formulas
// (bls_curve.h jac_dbl / jac_add / mul_by_xabs, templates over the coordinate field) are
// instantiated for r28::fe2 through the overload set below, found by argument-dependent lookup.
// Every operation returns a normalized, weakly reduced value (< 1.03 p), so each formula's
// inputs meet fe2_mul / fe2_sqr's bounds without bookkeeping; a product costs ~0.84 us per
// lane instead of the engine's ~1.18 (tools/ubench/r28_bench.hip).
#pragma once
#include "bls_curve.h"
#include "bls_field28.h"
#include "bls_r28_consts.h"

namespace gbls {
namespace r28 {

HD void f_add(fe2 &r, const fe2 &a, const fe2 &b) { fe2_add_r(r, a, b); }
HD void f_sub(fe2 &r, const fe2 &a, const fe2 &b) { fe2_sub_r(r, a, b); }
HD void f_mul(fe2 &r, const fe2 &a, const fe2 &b) { fe2_mul(r, a, b); }
HD void f_sqr(fe2 &r, const fe2 &a) { fe2_sqr(r, a); }
HD void f_dbl(fe2 &r, const fe2 &a) { fe2_add_r(r, a, a); }
HD void f_zero(fe2 &r) {
#pragma unroll
  for (int i = 0; i < 14; i++) r.c0.l[i] = r.c1.l[i] = 0;
}
HD void f_neg(fe2 &r, const fe2 &a) {
  fe2 z;
  f_zero(z);
  fe2_sub_r(r, z, a);
}
HD void f_one(fe2 &r) {
  r.c0 = K28_ONE;
#pragma unroll
  for (int i = 0; i < 14; i++) r.c1.l[i] = 0;
}
HD bool f_is_zero(const fe2 &a) { return is_zero(a.c0) && is_zero(a.c1); }

typedef jac<fe2> g2j28;

HD void g2j_in(g2j28 &r, const g2j &a) {
  from_fp(r.x.c0, a.x.c0);
  from_fp(r.x.c1, a.x.c1);
  from_fp(r.y.c0, a.y.c0);
  from_fp(r.y.c1, a.y.c1);
  from_fp(r.z.c0, a.z.c0);
  from_fp(r.z.c1, a.z.c1);
}
HD void g2j_out(g2j &r, const g2j28 &a) {
  to_fp(r.x.c0, a.x.c0);
  to_fp(r.x.c1, a.x.c1);
  to_fp(r.y.c0, a.y.c0);
  to_fp(r.y.c1, a.y.c1);
  to_fp(r.z.c0, a.z.c0);
  to_fp(r.z.c1, a.z.c1);
}
// psi(x, y, z) = (conj(x) cx, conj(y) cy, conj(z)) with cx = K28_PSI_CX1 u
HD void g2_psi28(g2j28 &r, const g2j28 &p) {
  fe2 t, c;
  t.c0 = p.x.c0;
  f_zero(c);
  sub_r(t.c1, c.c0, p.x.c1);  // conj(x)
  // (t0 + t1 u)(k u) = -t1 k + t0 k u
  fe n1;
  mul(n1, t.c1, K28_PSI_CX1);
  mul(r.x.c1, t.c0, K28_PSI_CX1);
  sub_r(r.x.c0, c.c0, n1);
  t.c0 = p.y.c0;
  sub_r(t.c1, c.c0, p.y.c1);  // conj(y)
  c.c0 = K28_PSI_CY0;
  c.c1 = K28_PSI_CY1;
  fe2_mul(r.y, t, c);
  r.z.c0 = p.z.c0;
  f_zero(c);
  sub_r(r.z.c1, c.c0, p.z.c1);
}
HD void g2_psi2_28(g2j28 &r, const g2j28 &p) {
  fe2_mul_fe(r.x, p.x, K28_PSI2_CX);
  fe2_mul_fe(r.y, p.y, K28_PSI2_CY);
  r.z = p.z;
}

// h_eff P, the sequence of clear_cofactor_g2 (bls_hash.h, Budroni-Pintore): host tests of
// the layer's G2 formulas (tests/native/host_harness.cpp)
HD void clear_cofactor28(g2j28 &r, const g2j28 &p) {
  g2j28 t1, t2, t3;
  mul_by_xabs(t1, p);
  jac_neg(t1, t1);  // t1 = [x]P
  g2_psi28(t2, p);
  jac_add(t2, t2, t1);  // t1 + psi(P)
  mul_by_xabs(t3, t2);
  jac_neg(t3, t3);  // t3 = [x](t1 + psi(P))
  jac_neg(t1, t1);
  jac_add(t3, t3, t1);  // - t1
  jac_dbl(t1, p);
  g2_psi2_28(t1, t1);
  jac_add(t3, t3, t1);  // + psi^2(2P)
  g2_psi28(t1, p);
  jac_neg(t1, t1);
  jac_add(t3, t3, t1);  // - psi(P)
  jac_neg(t1, p);
  jac_add(r, t3, t1);  // - P
}

}  // namespace r28
}  // namespace gbls
