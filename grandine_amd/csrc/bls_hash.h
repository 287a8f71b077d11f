// hash_to_G2 for the BLS12381G2_XMD:SHA-256_SSWU_RO_ suite (RFC 9380), the map
// blst's Hash_to_G2 applies to every signed message (bls/src/consts.rs:1 DST;
// bls/src/signature.rs:50-57,85-90,117-126; secret_key.rs:82-86).
//
// expand_message_xmd (SHA-256, 256 bytes) -> 2 x Fp2 -> simplified SWU on the
// 3-isogenous curve E2' -> 3-isogeny to E2 -> point addition -> cofactor clearing
// with the Budroni-Pintore endomorphism formula (equal to h_eff multiplication).
#pragma once
#include "bls_curve.h"

namespace gbls {

// ---------------------------------------------------------------- SHA-256
struct sha_state {
  uint32_t h[8];
};

HD uint32_t rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

HD void sha256_init(sha_state &s) {
  s.h[0] = 0x6a09e667u;
  s.h[1] = 0xbb67ae85u;
  s.h[2] = 0x3c6ef372u;
  s.h[3] = 0xa54ff53au;
  s.h[4] = 0x510e527fu;
  s.h[5] = 0x9b05688cu;
  s.h[6] = 0x1f83d9abu;
  s.h[7] = 0x5be0cd19u;
}

HD void sha256_compress(sha_state &s, const uint32_t (&blk)[16]) {
  const uint32_t K[64] = {
      0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u,
      0xab1c5ed5u, 0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu,
      0x9bdc06a7u, 0xc19bf174u, 0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu,
      0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau, 0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u,
      0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u, 0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu,
      0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u, 0xa2bfe8a1u, 0xa81a664bu,
      0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u, 0x19a4c116u,
      0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
      0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u,
      0xc67178f2u};
  uint32_t w[16];
#pragma unroll
  for (int i = 0; i < 16; i++) w[i] = blk[i];
  uint32_t a = s.h[0], b = s.h[1], c = s.h[2], d = s.h[3], e = s.h[4], f = s.h[5], g = s.h[6],
           h = s.h[7];
#pragma unroll
  for (int i = 0; i < 64; i++) {
    uint32_t wi;
    if (i < 16) {
      wi = w[i];
    } else {
      uint32_t w15 = w[(i - 15) & 15], w2 = w[(i - 2) & 15];
      uint32_t s0 = rotr(w15, 7) ^ rotr(w15, 18) ^ (w15 >> 3);
      uint32_t s1 = rotr(w2, 17) ^ rotr(w2, 19) ^ (w2 >> 10);
      wi = w[i & 15] + s0 + w[(i - 7) & 15] + s1;
      w[i & 15] = wi;
    }
    uint32_t S1 = rotr(e, 6) ^ rotr(e, 11) ^ rotr(e, 25);
    uint32_t ch = (e & f) ^ (~e & g);
    uint32_t t1 = h + S1 + ch + K[i] + wi;
    uint32_t S0 = rotr(a, 2) ^ rotr(a, 13) ^ rotr(a, 22);
    uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
    uint32_t t2 = S0 + mj;
    h = g;
    g = f;
    f = e;
    e = d + t1;
    d = c;
    c = b;
    b = a;
    a = t1 + t2;
  }
  s.h[0] += a;
  s.h[1] += b;
  s.h[2] += c;
  s.h[3] += d;
  s.h[4] += e;
  s.h[5] += f;
  s.h[6] += g;
  s.h[7] += h;
}

// A domain separation tag, <= 255 bytes, resident in device (or host) memory.
struct dst_ref {
  const uint8_t *p;
  uint32_t len;
};

// Byte source for the tail of b_0's input:  msg || I2OSP(256,2) || 0x00 || DST || len(DST)
// (the 64-byte Z_pad block is hashed separately), followed by SHA-256 padding.
struct b0_src {
  const uint8_t *msg;
  uint32_t mlen;
  dst_ref dst;
  uint32_t total;  // bytes of real data after Z_pad
  HD uint32_t byte(uint32_t i) const {
    if (i < mlen) return msg[i];
    i -= mlen;
    if (i < 3) return i == 0 ? 0x01 : 0x00;
    i -= 3;
    if (i < dst.len) return dst.p[i];
    if (i == dst.len) return dst.len;
    return 0;
  }
};

HD void sha_fill_block(uint32_t (&blk)[16], const b0_src &src, uint32_t base, uint32_t nbytes,
                       uint64_t bitlen, bool last) {
#pragma unroll
  for (int wi = 0; wi < 16; wi++) {
    uint32_t v = 0;
#pragma unroll
    for (int bi = 0; bi < 4; bi++) {
      uint32_t idx = base + 4 * wi + bi;
      uint32_t byte;
      if (idx < nbytes)
        byte = src.byte(idx);
      else if (idx == nbytes)
        byte = 0x80;
      else
        byte = 0;
      v = (v << 8) | byte;
    }
    blk[wi] = v;
  }
  if (last) {
    blk[14] = (uint32_t)(bitlen >> 32);
    blk[15] = (uint32_t)bitlen;
  }
}

// expand_message_xmd(msg, DST, 256): the 64 big-endian 32-bit words of the output go to
// sink(k, w) as 4 chunks of 16 (k = 0..3: b_(2k+1) || b_(2k+2)), so that every array here
// is indexed by constants (registers, no scratch).
template <class Sink>
HD void expand_message_xmd_256(const uint8_t *msg, uint32_t mlen, dst_ref dst, Sink &&sink) {
  sha_state s;
  sha256_init(s);
  uint32_t blk[16];
#pragma unroll
  for (int i = 0; i < 16; i++) blk[i] = 0;
  sha256_compress(s, blk);  // Z_pad (64 zero bytes)
  b0_src src{msg, mlen, dst, mlen + 3 + dst.len + 1};
  uint64_t bitlen = (uint64_t)(64 + src.total) * 8;
  uint32_t nblk = (src.total + 9 + 63) / 64;
  for (uint32_t b = 0; b < nblk; b++) {
    sha_fill_block(blk, src, 64 * b, src.total, bitlen, b + 1 == nblk);
    sha256_compress(s, blk);
  }
  uint32_t b0[8];
#pragma unroll
  for (int i = 0; i < 8; i++) b0[i] = s.h[i];
  // b_i = H((b_0 ^ b_{i-1}) || I2OSP(i,1) || DST || len(DST)),  b_1 uses b_{0} ^ 0 = b_0
  uint32_t prev[8];
#pragma unroll
  for (int i = 0; i < 8; i++) prev[i] = 0;
  uint32_t chunk[16];
  for (int bi = 1; bi <= 8; bi++) {
    // message: 32 bytes x || 1 byte i || dst || dstlen  = 33 + dst.len + 1 bytes
    uint32_t xw[8];
#pragma unroll
    for (int i = 0; i < 8; i++) xw[i] = b0[i] ^ prev[i];
    uint32_t mlen2 = 33 + dst.len + 1;
    uint32_t nb2 = (mlen2 + 9 + 63) / 64;
    uint64_t bl2 = (uint64_t)mlen2 * 8;
    sha256_init(s);
    for (uint32_t b = 0; b < nb2; b++) {
#pragma unroll
      for (int wi = 0; wi < 16; wi++) {
        uint32_t v = 0;
#pragma unroll
        for (int q = 0; q < 4; q++) {
          const uint32_t idx = 64 * b + 4 * wi + q;
          uint32_t byte;
          if (idx < 32) {
            uint32_t x = 0;  // xw[idx >> 2] by a select chain (idx is not a constant)
#pragma unroll
            for (int t = 0; t < 8; t++) x = (idx >> 2) == (uint32_t)t ? xw[t] : x;
            byte = (x >> (24 - 8 * (idx & 3))) & 0xff;
          } else if (idx == 32) {
            byte = (uint32_t)bi;
          } else if (idx < 33 + dst.len) {
            byte = dst.p[idx - 33];
          } else if (idx == 33 + dst.len) {
            byte = dst.len;
          } else if (idx == mlen2) {
            byte = 0x80;
          } else {
            byte = 0;
          }
          v = (v << 8) | byte;
        }
        blk[wi] = v;
      }
      if (b + 1 == nb2) {
        blk[14] = (uint32_t)(bl2 >> 32);
        blk[15] = (uint32_t)bl2;
      }
      sha256_compress(s, blk);
    }
#pragma unroll
    for (int i = 0; i < 8; i++) prev[i] = s.h[i];
    if (bi & 1) {
#pragma unroll
      for (int i = 0; i < 8; i++) chunk[i] = s.h[i];
    } else {
#pragma unroll
      for (int i = 0; i < 8; i++) chunk[8 + i] = s.h[i];
      sink((bi >> 1) - 1, chunk);
    }
  }
}
// the 64 output words in one array (host tests and tools)
HD void expand_message_xmd_256(uint32_t (&out)[64], const uint8_t *msg, uint32_t mlen, dst_ref dst) {
  expand_message_xmd_256(msg, mlen, dst, [&](int k, const uint32_t (&w)[16]) {
    for (int i = 0; i < 16; i++) out[16 * k + i] = w[i];
  });
}

// 64 big-endian bytes (16 BE words starting at w) mod p, in Montgomery form:
// v = hi * 2^256 + lo  ->  mont(v) = fp_mul(hi, 2^256 R^2) + fp_mul(lo, R^2)
HD void fp_from_be64_words(fp &r, const uint32_t *w) {
  fp hi, lo;
  fp_zero(hi);
  fp_zero(lo);
#pragma unroll
  for (int i = 0; i < 8; i++) {
    hi.l[i] = w[7 - i];
    lo.l[i] = w[15 - i];
  }
  fp a, b;
  fp_mul(a, hi, fp_const(k::R2_SHL256));
  fp_mul(b, lo, fp_const(k::R2));
  fp_add(r, a, b);
}

// ---------------------------------------------------------------- SSWU + isogeny
// fp2_sqrt_given_norm_root (bls_field.h) that also returns 1/nd for an nd != 0 in Fp,
// without an inversion: the exponentiation runs on delta nd^4 instead of delta,
//   t' = (delta nd^4)^((p-3)/4) = t nd^(p-3) = t / nd^2     (t = delta^((p-3)/4))
// so t = t' nd^2, chi = delta t^2 = +-1 (delta's quadratic character), 1/t = chi delta t
// and 1/nd = nd (t' / t) = chi nd t' t delta.  delta = 0 (only when a = 0) has no
// character; that case falls back to the binary-GCD inversion.
// The exponentiation a^((p-3)/4) is a policy (Pow) so that the latency-regime kernel can
// run it on a 16-lane row (bls_dfp.h) while the rest of the map stays per lane.
struct LanePow {
  HD void operator()(fp &r, const fp &a) const { fp_pow_pm3d4(r, a); }
};
template <class Pow>
HD void fp2_sqrt_norm_inv(fp2 &r, fp &ndinv, const fp2 &a, const fp &gamma, const fp &nd,
                          const Pow &pow) {
  fp delta, t, tp, x0, x0sq, tmp, nd2, u;
  fp_add(delta, a.c0, gamma);
  fp_half(delta, delta);
  if (fp_is_zero(delta)) {  // only when a1 == 0 and gamma == -a0
    fp_sub(delta, a.c0, gamma);
    fp_half(delta, delta);
  }
  fp_sqr(nd2, nd);
  fp_sqr(u, nd2);
  fp_mul(u, u, delta);     // delta nd^4
  pow(tp, u);              // t'
  fp_mul(t, tp, nd2);      // t
  fp_mul(x0, delta, t);
  fp_sqr(x0sq, x0);
  fp half_a1t;
  fp_mul(tmp, a.c1, t);
  fp_half(half_a1t, tmp);
  bool sq = fp_eq(x0sq, delta);  // chi = +1
  fp nh;
  fp_neg(nh, half_a1t);
  fp_sel(r.c0, sq, nh, x0);
  fp_sel(r.c1, sq, x0, half_a1t);
  if (fp_is_zero(delta)) {
    fp_inv(ndinv, nd);
    return;
  }
  fp_mul(u, nd, tp);
  fp_mul(u, u, x0);        // nd t' t delta
  fp_neg(tmp, u);
  fp_sel(ndinv, sq, tmp, u);
}

// Simplified SWU on E2': y^2 = x^3 + A'x + B' (RFC 9380 §6.6.2), inversion-free up to
// one final Fp2 inversion, returning a Jacobian point on E2'.
template <class Pow>
HD void map_to_curve_sswu(g2j &out, const fp2 &u, const Pow &pow) {
  const fp2 A = fp2_const(k::SSWU_A_C0, k::SSWU_A_C1);
  const fp2 B = fp2_const(k::SSWU_B_C0, k::SSWU_B_C1);
  const fp2 Z = fp2_const(k::SSWU_Z_C0, k::SSWU_Z_C1);
  fp2 u2, zu2, tv1, N, D, t;
  fp2_sqr(u2, u);
  fp2_mul(zu2, Z, u2);
  fp2_sqr(tv1, zu2);
  fp2_add(tv1, tv1, zu2);  // Z^2 u^4 + Z u^2
  // x1 = N/D = -B (tv1 + 1) / (A tv1);  tv1 == 0 -> x1 = B / (Z A)
  bool exc = fp2_is_zero(tv1);
  fp2 one;
  fp2_one(one);
  fp2_add(t, tv1, one);
  fp2_mul(N, fp2_const(k::SSWU_NEGB_C0, k::SSWU_NEGB_C1), t);
  fp2_mul(D, A, tv1);
  fp2_sel(N, exc, N, B);
  fp2_sel(D, exc, D, fp2_const(k::SSWU_ZA_C0, k::SSWU_ZA_C1));
  // U = N^3 + A N D^2 + B D^3;  gx1 = U / D^3, square-ness of gx1 == that of U D
  fp2 D2, D3, N2, U, a1;
  fp2_sqr(D2, D);
  fp2_mul(D3, D2, D);
  fp2_sqr(N2, N);
  fp2_mul(U, N2, N);
  fp2_mul(t, A, N);
  fp2_mul(t, t, D2);
  fp2_add(U, U, t);
  fp2_mul(t, B, D3);
  fp2_add(U, U, t);
  fp2_mul(a1, U, D);
  // norm and its Fp square root
  fp n, nt, gamma, g2;
  fp_sqr(n, a1.c0);
  fp_sqr(nt, a1.c1);
  fp_add(n, n, nt);
  pow(gamma, n);
  fp_mul(gamma, gamma, n);  // n^((p+1)/4)
  fp_sqr(g2, gamma);
  bool is_sq = fp_eq(g2, n);
  // x2 = Z u^2 x1, gx2 = (Z u^2)^3 gx1 -> U2 D = (Z u^2)^3 U D ; sqrt(N(.)) = N(u)^3 sqrt(-125) gamma
  fp2 zu2_3, a2;
  fp2_sqr(zu2_3, zu2);
  fp2_mul(zu2_3, zu2_3, zu2);
  fp2_mul(a2, zu2_3, a1);
  fp nu, nu3, gamma2;
  fp_sqr(nu, u.c0);
  fp_sqr(nt, u.c1);
  fp_add(nu, nu, nt);
  fp_sqr(nu3, nu);
  fp_mul(nu3, nu3, nu);
  fp_mul(gamma2, nu3, fp_const(k::SQRT_M125_M));
  fp_mul(gamma2, gamma2, gamma);
  fp2 a, Nsel, s;
  fp2_sel(a, is_sq, a2, a1);
  fp gsel;
  fp_sel(gsel, is_sq, gamma2, gamma);
  fp2 Nx2;
  fp2_mul(Nx2, zu2, N);
  fp2_sel(Nsel, is_sq, Nx2, N);
  // s^2 = U_sel D, and 1/N(D) from the same exponentiation (fp2_sqrt_norm_inv)
  fp nd, ndt, ndinv;
  fp_sqr(nd, D.c0);
  fp_sqr(ndt, D.c1);
  fp_add(nd, nd, ndt);
  fp2_sqrt_norm_inv(s, ndinv, a, gsel, nd, pow);
  // affine: x = Nsel / D, y = s / D^2  (sgn0 needs the affine y); 1/D = conj(D) / N(D)
  fp2 Di, Di2, x, y;
  fp2_conj(Di, D);
  fp2_mul_fp(Di, Di, ndinv);
  fp2_sqr(Di2, Di);
  fp2_mul(x, Nsel, Di);
  fp2_mul(y, s, Di2);
  if (fp2_sgn0(u) != fp2_sgn0(y)) fp2_neg(y, y);
  out.x = x;
  out.y = y;
  fp2_one(out.z);
}

// 3-isogeny E2' -> E2 on an affine-in-Jacobian (z = 1) input; Jacobian output
// with Z = xd * yd:  X = xn xd yd^2,  Y = y yn xd^3 yd^2.
HD void iso_map_g2(g2j &out, const g2j &in) {
  const fp2 &x = in.x;
  fp2 x2, x3, xn, xd, yn, yd, t;
  fp2_sqr(x2, x);
  fp2_mul(x3, x2, x);
  // xn = k13 x^3 + k12 x^2 + k11 x + k10
  fp2_mul(xn, fp2_const(k::ISO_XNUM3_C0, k::ISO_XNUM3_C1), x3);
  fp2_mul(t, fp2_const(k::ISO_XNUM2_C0, k::ISO_XNUM2_C1), x2);
  fp2_add(xn, xn, t);
  fp2_mul(t, fp2_const(k::ISO_XNUM1_C0, k::ISO_XNUM1_C1), x);
  fp2_add(xn, xn, t);
  fp2_add(xn, xn, fp2_const(k::ISO_XNUM0_C0, k::ISO_XNUM0_C1));
  // xd = x^2 + k21 x + k20
  fp2_mul(t, fp2_const(k::ISO_XDEN1_C0, k::ISO_XDEN1_C1), x);
  fp2_add(xd, x2, t);
  fp2_add(xd, xd, fp2_const(k::ISO_XDEN0_C0, k::ISO_XDEN0_C1));
  // yn = k33 x^3 + k32 x^2 + k31 x + k30
  fp2_mul(yn, fp2_const(k::ISO_YNUM3_C0, k::ISO_YNUM3_C1), x3);
  fp2_mul(t, fp2_const(k::ISO_YNUM2_C0, k::ISO_YNUM2_C1), x2);
  fp2_add(yn, yn, t);
  fp2_mul(t, fp2_const(k::ISO_YNUM1_C0, k::ISO_YNUM1_C1), x);
  fp2_add(yn, yn, t);
  fp2_add(yn, yn, fp2_const(k::ISO_YNUM0_C0, k::ISO_YNUM0_C1));
  // yd = x^3 + k42 x^2 + k41 x + k40
  fp2_mul(t, fp2_const(k::ISO_YDEN2_C0, k::ISO_YDEN2_C1), x2);
  fp2_add(yd, x3, t);
  fp2_mul(t, fp2_const(k::ISO_YDEN1_C0, k::ISO_YDEN1_C1), x);
  fp2_add(yd, yd, t);
  fp2_add(yd, yd, fp2_const(k::ISO_YDEN0_C0, k::ISO_YDEN0_C1));
  // exceptional (xd or yd zero): the image is the identity, selected after the arithmetic
  // (an early return made the compiler keep the output in scratch memory)
  const bool exc = fp2_is_zero(xd) || fp2_is_zero(yd);
  fp2 yd2, xd3;
  fp2_sqr(yd2, yd);
  fp2_mul(out.x, xn, xd);
  fp2_mul(out.x, out.x, yd2);
  fp2_sqr(xd3, xd);
  fp2_mul(xd3, xd3, xd);
  fp2_mul(t, in.y, yn);
  fp2_mul(t, t, xd3);
  fp2_mul(out.y, t, yd2);
  fp2_mul(out.z, xd, yd);
  if (exc) jac_set_inf(out);
}

// h_eff P = [x^2-x-1]P + [x-1]psi(P) + psi^2(2P)  (Budroni-Pintore; RFC 9380 G.3):
//   t1 = [x]P;  t2 = [x](t1 + psi(P));  h = t2 - t1 + psi^2(2P) - psi(P) - P
// ordered so that at most three Jacobian points are live at once.
HD void clear_cofactor_g2(g2j &r, const g2j &p) {
  g2j t1, t2, t3;
  mul_by_xabs(t1, p);
  jac_neg(t1, t1);        // t1 = [x]P
  g2_psi(t2, p);
  jac_add(t2, t2, t1);    // t1 + psi(P)
  mul_by_xabs(t3, t2);
  jac_neg(t3, t3);        // t3 = [x](t1 + psi(P))
  jac_neg(t1, t1);
  jac_add(t3, t3, t1);    // - t1
  jac_dbl(t1, p);
  g2_psi2(t1, t1);
  jac_add(t3, t3, t1);    // + psi^2(2P)
  g2_psi(t1, p);
  jac_neg(t1, t1);
  jac_add(t3, t3, t1);    // - psi(P)
  jac_neg(t1, p);
  jac_add(r, t3, t1);     // - P
}

// hash_to_field (RFC 9380 §5.2, count = 2, m = 2, L = 64): msg -> u[0], u[1] in Fp2
HD void hash_to_field_g2(fp2 (&u)[2], const uint8_t *msg, uint32_t mlen, dst_ref dst) {
  fp e0, e1, e2, e3;
  fp_zero(e0);
  fp_zero(e1);
  fp_zero(e2);
  fp_zero(e3);
  expand_message_xmd_256(msg, mlen, dst, [&](int k, const uint32_t (&w)[16]) {
    fp v;
    fp_from_be64_words(v, w);
    // k is not a constant: selects keep the four elements in registers
    fp_sel(e0, k == 0, e0, v);  // (c ? b : a)
    fp_sel(e1, k == 1, e1, v);
    fp_sel(e2, k == 2, e2, v);
    fp_sel(e3, k == 3, e3, v);
  });
  u[0].c0 = e0;
  u[0].c1 = e1;
  u[1].c0 = e2;
  u[1].c1 = e3;
}
// map_to_curve (SSWU + 3-isogeny) of one field element -> Jacobian point on E2
template <class Pow>
HD void map_to_g2(g2j &q, const fp2 &u, const Pow &pow) {
  g2j m;
  map_to_curve_sswu(m, u, pow);
  iso_map_g2(q, m);
}
HD void map_to_g2(g2j &q, const fp2 &u) { map_to_g2(q, u, LanePow()); }
// hash_to_curve(msg) with DST, result as a Jacobian point on E2 (in G2).  The device
// pipeline runs the same three stages as separate kernels (k_h2c_*).
HD void hash_to_g2(g2j &r, const uint8_t *msg, uint32_t mlen, dst_ref dst) {
  fp2 u[2];
  hash_to_field_g2(u, msg, mlen, dst);
  g2j q0, q1;
  map_to_g2(q0, u[0]);
  map_to_g2(q1, u[1]);
  jac_add(q0, q0, q1);
  clear_cofactor_g2(r, q0);
}

}  // namespace gbls
