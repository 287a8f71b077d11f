"""BLS12-381 CPU oracle (pure Python ints) -- TEST INFRASTRUCTURE ONLY.

This module is the checker for the MI355X engine in ``grandine_amd``.  Only
``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
may import it; the product path never does.

It restates, from the published algorithms, what the reference's hot path
delegates to blst 0.3.11 (a crates.io dependency, not vendored in
/root/reference -- see SURVEY.md §0/§8c):

* field tower Fp / Fp2 = Fp[u]/(u^2+1) / Fp12 = Fp2[w]/(w^6 - (1+u));
* G1 (E: y^2 = x^3 + 4) and G2 (E': y^2 = x^3 + 4(1+u));
* ZCash point compression as used by ``PublicKey``/``Signature``
  (``bls/src/public_key.rs:9-31``, ``bls/src/signature.rs:29-45``);
* RFC 9380 hash_to_curve, suite BLS12381G2_XMD:SHA-256_SSWU_RO_ with the
  Ethereum POP DST (``bls/src/consts.rs:1``);
* optimal-ate pairing (Miller loop over |x| = 0xd201000000010000, x < 0) and
  final exponentiation by (p^12 - 1)/r, computed textbook-style;
* blst-semantics wrappers for ``Signature::verify`` (``signature.rs:47-60``),
  ``Signature::fast_aggregate_verify`` (``signature.rs:77-93``),
  ``Signature::multi_verify`` (``signature.rs:95-129``) and
  ``PublicKey::aggregate`` (``public_key.rs:34-55``).

Pinning: interop keygen KATs (``interop/src/lib.rs:119-178``), the EIP-2335
pubkey (``eip_2335/src/lib.rs:505,552``), the KZG trusted setup
(``kzg_utils/src/trusted_setup.txt``), algebraic self-checks, and RFC 9380
J.10.1 vectors recalled from memory (flagged in tests/golden).  Everything is
written for clarity, not speed; it is NOT constant time.
"""

from __future__ import annotations

import hashlib

# ---------------------------------------------------------------------------
# Parameters (each is asserted in tests/test_oracle.py)
# ---------------------------------------------------------------------------
P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
X_ABS = 0xD201000000010000  # |x|, x is negative
X = -X_ABS
DST_POP = b"BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_"  # bls/src/consts.rs:1

# BLST_ERROR codes (blst bindings; mirrored by include/grandine_bls_gpu.h)
SUCCESS, BAD_ENCODING, POINT_NOT_ON_CURVE, POINT_NOT_IN_GROUP = 0, 1, 2, 3
AGGR_TYPE_MISMATCH, VERIFY_FAIL, PK_IS_INFINITY, BAD_SCALAR = 4, 5, 6, 7


# ---------------------------------------------------------------------------
# Fp
# ---------------------------------------------------------------------------
def fp_inv(a: int) -> int:
    return pow(a, P - 2, P)


def fp_sqrt(a: int):
    """Return a square root of a mod p, or None.  p = 3 mod 4."""
    a %= P
    y = pow(a, (P + 1) // 4, P)
    return y if y * y % P == a else None


def fp_is_square(a: int) -> bool:
    a %= P
    return a == 0 or pow(a, (P - 1) // 2, P) == 1


def fp_sgn0(a: int) -> int:  # RFC 9380 §4.1 (parity)
    return a % P & 1


def fp_lex_largest(a: int) -> bool:  # ZCash serialization sort flag
    return a % P > (P - 1) // 2


# ---------------------------------------------------------------------------
# Fp2 = Fp[u]/(u^2 + 1), elements are tuples (c0, c1)
# ---------------------------------------------------------------------------
F2_ZERO = (0, 0)
F2_ONE = (1, 0)
XI = (1, 1)  # non-residue 1+u used for the twist and the tower


def f2(a, b=0):
    return (a % P, b % P)


def f2_add(a, b):
    return ((a[0] + b[0]) % P, (a[1] + b[1]) % P)


def f2_sub(a, b):
    return ((a[0] - b[0]) % P, (a[1] - b[1]) % P)


def f2_neg(a):
    return ((-a[0]) % P, (-a[1]) % P)


def f2_mul(a, b):
    return ((a[0] * b[0] - a[1] * b[1]) % P, (a[0] * b[1] + a[1] * b[0]) % P)


def f2_sqr(a):
    return f2_mul(a, a)


def f2_muls(a, s: int):
    return (a[0] * s % P, a[1] * s % P)


def f2_conj(a):
    return (a[0], (-a[1]) % P)


def f2_inv(a):
    n = (a[0] * a[0] + a[1] * a[1]) % P
    ni = fp_inv(n)
    return (a[0] * ni % P, (-a[1]) * ni % P)


def f2_pow(a, e: int):
    r = F2_ONE
    b = a
    while e:
        if e & 1:
            r = f2_mul(r, b)
        b = f2_mul(b, b)
        e >>= 1
    return r


def f2_is_zero(a) -> bool:
    return a[0] % P == 0 and a[1] % P == 0


def f2_is_square(a) -> bool:
    # a is a square in Fp2 iff its norm is a square in Fp
    return fp_is_square(a[0] * a[0] + a[1] * a[1])


def f2_sqrt(a):
    """A square root in Fp2 (complex method), or None."""
    a0, a1 = a[0] % P, a[1] % P
    if a1 == 0:
        s = fp_sqrt(a0)
        if s is not None:
            return (s, 0)
        s = fp_sqrt(-a0 % P)
        return (0, s) if s is not None else None
    gamma = fp_sqrt(a0 * a0 + a1 * a1)
    if gamma is None:
        return None
    inv2 = (P + 1) // 2
    delta = (a0 + gamma) * inv2 % P
    x0 = fp_sqrt(delta)
    if x0 is None:
        delta = (a0 - gamma) * inv2 % P
        x0 = fp_sqrt(delta)
        if x0 is None:
            return None
    x1 = a1 * fp_inv(2 * x0) % P
    r = (x0, x1)
    return r if f2_sqr(r) == (a0, a1) else None


def f2_sgn0(a) -> int:  # RFC 9380 §4.1, m = 2
    s0 = a[0] % 2
    z0 = a[0] == 0
    s1 = a[1] % 2
    return s0 | (z0 & s1)


def f2_lex_largest(a) -> bool:  # ZCash: compare c1 first, then c0
    if a[1] != 0:
        return fp_lex_largest(a[1])
    return fp_lex_largest(a[0])


# ---------------------------------------------------------------------------
# Fp12 = Fp2[w]/(w^6 - XI), elements are lists of 6 Fp2 coefficients
# ---------------------------------------------------------------------------
def f12_one():
    return [F2_ONE] + [F2_ZERO] * 5


def f12_mul(a, b):
    t = [F2_ZERO] * 11
    for i in range(6):
        ai = a[i]
        if ai == F2_ZERO:
            continue
        for j in range(6):
            if b[j] == F2_ZERO:
                continue
            t[i + j] = f2_add(t[i + j], f2_mul(ai, b[j]))
    out = t[:6]
    for k in range(6, 11):
        out[k - 6] = f2_add(out[k - 6], f2_mul(t[k], XI))
    return out


def f12_sqr(a):
    return f12_mul(a, a)


def f12_conj(a):
    """a^(p^6): w -> -w."""
    return [c if i % 2 == 0 else f2_neg(c) for i, c in enumerate(a)]


def f12_eq(a, b) -> bool:
    return all(x == y for x, y in zip(a, b))


def f12_is_one(a) -> bool:
    return f12_eq(a, f12_one())


# Frobenius: (sum c_i w^i)^p = sum conj(c_i) * XI^(i(p-1)/6) w^i
_FROB_G = [f2_pow(XI, i * (P - 1) // 6) for i in range(6)]


def f12_frob(a):
    return [f2_mul(f2_conj(c), _FROB_G[i]) for i, c in enumerate(a)]


def _f6_from_even(a):
    """Even part of an Fp12 element viewed in Fp6 = Fp2[v]/(v^3 - XI), v = w^2."""
    return (a[0], a[2], a[4])


def _f6_mul(a, b):
    t = [F2_ZERO] * 5
    for i in range(3):
        for j in range(3):
            t[i + j] = f2_add(t[i + j], f2_mul(a[i], b[j]))
    return (
        f2_add(t[0], f2_mul(t[3], XI)),
        f2_add(t[1], f2_mul(t[4], XI)),
        t[2],
    )


def _f6_inv(a):
    a0, a1, a2 = a
    c0 = f2_sub(f2_sqr(a0), f2_mul(XI, f2_mul(a1, a2)))
    c1 = f2_sub(f2_mul(XI, f2_sqr(a2)), f2_mul(a0, a1))
    c2 = f2_sub(f2_sqr(a1), f2_mul(a0, a2))
    t = f2_add(f2_mul(a0, c0), f2_mul(XI, f2_add(f2_mul(a2, c1), f2_mul(a1, c2))))
    ti = f2_inv(t)
    return (f2_mul(c0, ti), f2_mul(c1, ti), f2_mul(c2, ti))


def f12_inv(a):
    """a^-1 = conj(a) / (a * conj(a)); a*conj(a) lies in Fp6 (even powers of w)."""
    c = f12_conj(a)
    n = f12_mul(a, c)
    assert all(f2_is_zero(n[i]) for i in (1, 3, 5))
    ni = _f6_inv(_f6_from_even(n))
    ni12 = [ni[0], F2_ZERO, ni[1], F2_ZERO, ni[2], F2_ZERO]
    return f12_mul(c, ni12)


def f12_pow(a, e: int):
    r = f12_one()
    b = a
    while e:
        if e & 1:
            r = f12_mul(r, b)
        b = f12_sqr(b)
        e >>= 1
    return r


# ---------------------------------------------------------------------------
# Generic short-Weierstrass arithmetic (affine, None = infinity)
# ---------------------------------------------------------------------------
class _Field:
    def __init__(self, add, sub, mul, inv, neg, zero, one, eq):
        self.add, self.sub, self.mul, self.inv, self.neg = add, sub, mul, inv, neg
        self.zero, self.one, self.eq = zero, one, eq


FP = _Field(
    lambda a, b: (a + b) % P,
    lambda a, b: (a - b) % P,
    lambda a, b: a * b % P,
    fp_inv,
    lambda a: (-a) % P,
    0,
    1,
    lambda a, b: a % P == b % P,
)
FP2 = _Field(f2_add, f2_sub, f2_mul, f2_inv, f2_neg, F2_ZERO, F2_ONE, lambda a, b: a == b)

B1 = 4
B2 = (4, 4)


def _on_curve(F, b, pt) -> bool:
    if pt is None:
        return True
    x, y = pt
    return F.eq(F.mul(y, y), F.add(F.mul(F.mul(x, x), x), b))


def _add(F, p1, p2):
    if p1 is None:
        return p2
    if p2 is None:
        return p1
    x1, y1 = p1
    x2, y2 = p2
    if F.eq(x1, x2):
        if F.eq(y1, F.neg(y2)):
            return None
        # doubling
        three_x2 = F.mul(F.add(F.add(x1, x1), x1), x1)
        lam = F.mul(three_x2, F.inv(F.add(y1, y1)))
    else:
        lam = F.mul(F.sub(y2, y1), F.inv(F.sub(x2, x1)))
    x3 = F.sub(F.sub(F.mul(lam, lam), x1), x2)
    y3 = F.sub(F.mul(lam, F.sub(x1, x3)), y1)
    return (x3, y3)


def _neg(F, pt):
    return None if pt is None else (pt[0], F.neg(pt[1]))


def _mul(F, pt, k: int):
    if k < 0:
        return _mul(F, _neg(F, pt), -k)
    acc = None
    add = pt
    while k:
        if k & 1:
            acc = _add(F, acc, add)
        add = _add(F, add, add)
        k >>= 1
    return acc


G1_GEN = (
    0x17F1D3A73197D7942695638C4FA9AC0FC3688C4F9774B905A14E3A3F171BAC586C55E83FF97A1AEFFB3AF00ADB22C6BB,
    0x08B3F481E3AAA0F1A09E30ED741D8AE4FCF5E095D5D00AF600DB18CB2C04B3EDD03CC744A2888AE40CAA232946C5E7E1,
)
G2_GEN = (
    (
        0x024AA2B2F08F0A91260805272DC51051C6E47AD4FA403B02B4510B647AE3D1770BAC0326A805BBEFD48056C8C121BDB8,
        0x13E02B6052719F607DACD3A088274F65596BD0D09920B61AB5DA61BBDC7F5049334CF11213945D57E5AC7D055D042B7E,
    ),
    (
        0x0CE5D527727D6E118CC9CDC6DA2E351AADFD9BAA8CBDD3A76D429A695160D12C923AC9CC3BACA289E193548608B82801,
        0x0606C4A02EA734CC32ACD2B02BC28B99CB3E287E85A763AF267492AB572E99AB3F370D275CEC1DA1AAA9075FF05F79BE,
    ),
)


def g1_add(a, b):
    return _add(FP, a, b)


def g1_neg(a):
    return _neg(FP, a)


def g1_mul(a, k):
    return _mul(FP, a, k)


def g1_on_curve(a):
    return _on_curve(FP, B1, a)


def g2_add(a, b):
    return _add(FP2, a, b)


def g2_neg(a):
    return _neg(FP2, a)


def g2_mul(a, k):
    return _mul(FP2, a, k)


def g2_on_curve(a):
    return _on_curve(FP2, B2, a)


def g1_in_group(a) -> bool:
    """Textbook membership: [r]a == O (blst uses an endomorphism test)."""
    return g1_on_curve(a) and g1_mul(a, R) is None


def g2_in_group(a) -> bool:
    return g2_on_curve(a) and g2_mul(a, R) is None


# ---------------------------------------------------------------------------
# Serialization (ZCash format, big endian; blst_p1_uncompress / p2_uncompress)
# ---------------------------------------------------------------------------
def g1_compress(pt) -> bytes:
    if pt is None:
        return bytes([0xC0]) + bytes(47)
    x, y = pt
    b = bytearray(x.to_bytes(48, "big"))
    b[0] |= 0x80
    if fp_lex_largest(y):
        b[0] |= 0x20
    return bytes(b)


def g1_decompress(data: bytes):
    """-> (status, point).  Mirrors blst POINTonE1_Uncompress_Z."""
    if len(data) != 48:
        return BAD_ENCODING, None
    b0 = data[0]
    if not b0 & 0x80:
        return BAD_ENCODING, None
    if b0 & 0x40:
        if (b0 & 0x3F) == 0 and not any(data[1:]):
            return SUCCESS, None
        return BAD_ENCODING, None
    x = int.from_bytes(bytes([b0 & 0x1F]) + data[1:], "big")
    if x >= P:
        return BAD_ENCODING, None
    y = fp_sqrt(x * x * x + B1)
    if y is None:
        return POINT_NOT_ON_CURVE, None
    if fp_lex_largest(y) != bool(b0 & 0x20):
        y = P - y
    if x == 0:  # (0, +-2) has order 3
        return POINT_NOT_IN_GROUP, None
    return SUCCESS, (x, y)


def g2_compress(pt) -> bytes:
    if pt is None:
        return bytes([0xC0]) + bytes(95)
    x, y = pt
    b = bytearray(x[1].to_bytes(48, "big") + x[0].to_bytes(48, "big"))
    b[0] |= 0x80
    if f2_lex_largest(y):
        b[0] |= 0x20
    return bytes(b)


def g2_decompress(data: bytes):
    """-> (status, point).  Mirrors blst POINTonE2_Uncompress_Z (on-curve only)."""
    if len(data) != 96:
        return BAD_ENCODING, None
    b0 = data[0]
    if not b0 & 0x80:
        return BAD_ENCODING, None
    if b0 & 0x40:
        if (b0 & 0x3F) == 0 and not any(data[1:]):
            return SUCCESS, None
        return BAD_ENCODING, None
    x1 = int.from_bytes(bytes([b0 & 0x1F]) + data[1:48], "big")
    x0 = int.from_bytes(data[48:], "big")
    if x1 >= P or x0 >= P:
        return BAD_ENCODING, None
    x = (x0, x1)
    y = f2_sqrt(f2_add(f2_mul(f2_sqr(x), x), B2))
    if y is None:
        return POINT_NOT_ON_CURVE, None
    if f2_lex_largest(y) != bool(b0 & 0x20):
        y = f2_neg(y)
    return SUCCESS, (x, y)


# ---------------------------------------------------------------------------
# Hash to G2: RFC 9380, BLS12381G2_XMD:SHA-256_SSWU_RO_
# ---------------------------------------------------------------------------
def expand_message_xmd(msg: bytes, dst: bytes, len_in_bytes: int) -> bytes:
    """RFC 9380 §5.3.1 with H = SHA-256 (b_in_bytes 32, s_in_bytes 64)."""
    b_in, s_in = 32, 64
    ell = (len_in_bytes + b_in - 1) // b_in
    assert ell <= 255 and len(dst) <= 255
    dst_prime = dst + bytes([len(dst)])
    msg_prime = bytes(s_in) + msg + len_in_bytes.to_bytes(2, "big") + b"\x00" + dst_prime
    b0 = hashlib.sha256(msg_prime).digest()
    bi = hashlib.sha256(b0 + b"\x01" + dst_prime).digest()
    out = [bi]
    for i in range(2, ell + 1):
        bi = hashlib.sha256(bytes(x ^ y for x, y in zip(b0, bi)) + bytes([i]) + dst_prime).digest()
        out.append(bi)
    return b"".join(out)[:len_in_bytes]


def hash_to_field_fp2(msg: bytes, dst: bytes, count: int = 2):
    """RFC 9380 §5.2, m = 2, L = 64."""
    L = 64
    uniform = expand_message_xmd(msg, dst, count * 2 * L)
    out = []
    for i in range(count):
        e = []
        for j in range(2):
            off = L * (j + i * 2)
            e.append(int.from_bytes(uniform[off : off + L], "big") % P)
        out.append((e[0], e[1]))
    return out


# SSWU on E2': y^2 = x^3 + A' x + B'
SSWU_A = (0, 240)
SSWU_B = (1012, 1012)
SSWU_Z = f2(-2, -1)


def map_to_curve_sswu(u):
    """RFC 9380 §6.6.2 (straight-line, non-constant-time restatement)."""
    A, B, Z = SSWU_A, SSWU_B, SSWU_Z
    u2 = f2_sqr(u)
    zu2 = f2_mul(Z, u2)
    tv1 = f2_add(f2_sqr(zu2), zu2)  # Z^2 u^4 + Z u^2
    if f2_is_zero(tv1):
        x1 = f2_mul(B, f2_inv(f2_mul(Z, A)))
    else:
        x1 = f2_mul(f2_mul(f2_neg(B), f2_inv(A)), f2_add(F2_ONE, f2_inv(tv1)))
    gx1 = f2_add(f2_add(f2_mul(f2_sqr(x1), x1), f2_mul(A, x1)), B)
    if f2_is_square(gx1):
        x, y = x1, f2_sqrt(gx1)
    else:
        x = f2_mul(zu2, x1)
        gx2 = f2_add(f2_add(f2_mul(f2_sqr(x), x), f2_mul(A, x)), B)
        y = f2_sqrt(gx2)
    assert y is not None
    if f2_sgn0(u) != f2_sgn0(y):
        y = f2_neg(y)
    return (x, y)


def _h(s: str) -> int:
    return int(s, 16)


_PM = P  # shorthand for "p - k" constants below
# RFC 9380 Appendix E.3 (3-isogeny E2' -> E2).  Recalled constants; validated in
# tests by (i) iso(E2') lands on E2 and (ii) iso is a group homomorphism.
ISO_XNUM = [
    (_h("5c759507e8e333ebb5b7a9a47d7ed8532c52d39fd3a042a88b58423c50ae15d5c2638e343d9c71c6238aaaaaaaa97d6"),
     _h("5c759507e8e333ebb5b7a9a47d7ed8532c52d39fd3a042a88b58423c50ae15d5c2638e343d9c71c6238aaaaaaaa97d6")),
    (0, _h("11560bf17baa99bc32126fced787c88f984f87adf7ae0c7f9a208c6b4f20a4181472aaa9cb8d555526a9ffffffffc71a")),
    (_h("11560bf17baa99bc32126fced787c88f984f87adf7ae0c7f9a208c6b4f20a4181472aaa9cb8d555526a9ffffffffc71e"),
     _h("8ab05f8bdd54cde190937e76bc3e447cc27c3d6fbd7063fcd104635a790520c0a395554e5c6aaaa9354ffffffffe38d")),
    (_h("171d6541fa38ccfaed6dea691f5fb614cb14b4e7f4e810aa22d6108f142b85757098e38d0f671c7188e2aaaaaaaa5ed1"), 0),
]
ISO_XDEN = [f2(0, -72), f2(12, -12), F2_ONE]
ISO_YNUM = [
    (_h("1530477c7ab4113b59a4c18b076d11930f7da5d4a07f649bf54439d87d27e500fc8c25ebf8c92f6812cfc71c71c6d706"),
     _h("1530477c7ab4113b59a4c18b076d11930f7da5d4a07f649bf54439d87d27e500fc8c25ebf8c92f6812cfc71c71c6d706")),
    (0, _h("5c759507e8e333ebb5b7a9a47d7ed8532c52d39fd3a042a88b58423c50ae15d5c2638e343d9c71c6238aaaaaaaa97be")),
    (_h("11560bf17baa99bc32126fced787c88f984f87adf7ae0c7f9a208c6b4f20a4181472aaa9cb8d555526a9ffffffffc71c"),
     _h("8ab05f8bdd54cde190937e76bc3e447cc27c3d6fbd7063fcd104635a790520c0a395554e5c6aaaa9354ffffffffe38f")),
    (_h("124c9ad43b6cf79bfbf7043de3811ad0761b0f37a1e26286b0e977c69aa274524e79097a56dc4bd9e1b371c71c718b10"), 0),
]
ISO_YDEN = [f2(-432, -432), f2(0, -216), f2(18, -18), F2_ONE]


def _poly(coeffs, x):
    acc = F2_ZERO
    for c in reversed(coeffs):
        acc = f2_add(f2_mul(acc, x), c)
    return acc


def iso_map_g2(pt):
    """E2' -> E2 (RFC 9380 §6.6.3 / Appendix E.3)."""
    if pt is None:
        return None
    x, y = pt
    xd = _poly(ISO_XDEN, x)
    yd = _poly(ISO_YDEN, x)
    if f2_is_zero(xd) or f2_is_zero(yd):
        return None
    xo = f2_mul(_poly(ISO_XNUM, x), f2_inv(xd))
    yo = f2_mul(y, f2_mul(_poly(ISO_YNUM, x), f2_inv(yd)))
    return (xo, yo)


# Effective cofactor for G2 (RFC 9380 §8.8.2).  Recalled; tests cross-check it
# against the Budroni-Pintore formula below and against [r]h_eff P == O.
H_EFF_G2 = _h(
    "bc69f08f2ee75b3584c6a0ea91b352888e2a8e9145ad7689986ff031508ffe1329c2f178731db956d82bf015d1212b02"
    "ec0ec69d7477c1ae954cbc06689f6a359894c0adebbf6b4e8020005aaa95551"
)

# psi = untwist -> Frobenius -> twist:  (x, y) -> (conj(x) c_x, conj(y) c_y)
PSI_CX = f2_inv(f2_pow(XI, (P - 1) // 3))
PSI_CY = f2_inv(f2_pow(XI, (P - 1) // 2))


def g2_psi(pt):
    if pt is None:
        return None
    x, y = pt
    return (f2_mul(f2_conj(x), PSI_CX), f2_mul(f2_conj(y), PSI_CY))


def clear_cofactor_g2(pt):
    """h_eff * P (RFC 9380 §8.8.2), done as a plain scalar multiplication."""
    return g2_mul(pt, H_EFF_G2)


def clear_cofactor_g2_bp(pt):
    """Budroni-Pintore: [x^2-x-1]P + [x-1]psi(P) + psi^2(2P) (equals h_eff*P)."""
    t1 = g2_mul(pt, X * X - X - 1)
    t2 = g2_mul(g2_psi(pt), X - 1)
    t3 = g2_psi(g2_psi(g2_add(pt, pt)))
    return g2_add(g2_add(t1, t2), t3)


def hash_to_g2(msg: bytes, dst: bytes = DST_POP):
    u0, u1 = hash_to_field_fp2(msg, dst, 2)
    q0 = iso_map_g2(map_to_curve_sswu(u0))
    q1 = iso_map_g2(map_to_curve_sswu(u1))
    return clear_cofactor_g2(g2_add(q0, q1))


# ---------------------------------------------------------------------------
# Pairing
# ---------------------------------------------------------------------------
def _line_sparse(lam, xt, yt, xp, yp):
    """w^3 * (yP - yT - lambda (xP - xT)) for T on the twist, P in G1.

    With psi(x', y') = (x' w^-2, y' w^-3), the untwisted slope is lambda' w^-1,
    so the scaled line is  (lambda' x'_T - y'_T) + (-lambda' xP) w^2 + yP w^3.
    The w^3 factor lies in a proper subfield and dies in the final exponentiation.
    """
    c0 = f2_sub(f2_mul(lam, xt), yt)
    c2 = f2_neg(f2_muls(lam, xp))
    c3 = (yp % P, 0)
    return [c0, F2_ZERO, c2, c3, F2_ZERO, F2_ZERO]


def miller_loop(p1, q2):
    """f_{|x|,Q}(P), conjugated because x < 0.  p1 in G1 (affine), q2 in G2."""
    if p1 is None or q2 is None:
        return f12_one()
    xp, yp = p1
    f = f12_one()
    t = q2
    for bit in bin(X_ABS)[3:]:
        xt, yt = t
        lam = f2_mul(f2_muls(f2_sqr(xt), 3), f2_inv(f2_add(yt, yt)))
        f = f12_mul(f12_sqr(f), _line_sparse(lam, xt, yt, xp, yp))
        t = g2_add(t, t)
        if bit == "1":
            xt, yt = t
            xq, yq = q2
            lam = f2_mul(f2_sub(yt, yq), f2_inv(f2_sub(xt, xq)))
            f = f12_mul(f, _line_sparse(lam, xt, yt, xp, yp))
            t = g2_add(t, q2)
    return f12_conj(f)


FINAL_EXP_HARD = (P**4 - P**2 + 1) // R


def final_exp(f):
    """f^((p^12-1)/r), textbook: easy part via conj/inverse/Frobenius, hard part by pow."""
    f = f12_mul(f12_conj(f), f12_inv(f))  # ^(p^6 - 1)
    f = f12_mul(f12_frob(f12_frob(f)), f)  # ^(p^2 + 1)
    return f12_pow(f, FINAL_EXP_HARD)


def pairing(p1, q2):
    return final_exp(miller_loop(p1, q2))


# ---------------------------------------------------------------------------
# Keys and signatures (blst min_pk semantics)
# ---------------------------------------------------------------------------
def sk_from_bytes(b: bytes):
    """-> (status, sk).  blst SecretKey::from_bytes: 32 B big endian, 0 < sk < r."""
    if len(b) != 32:
        return BAD_ENCODING, None
    k = int.from_bytes(b, "big")
    if k == 0 or k >= R:
        return BAD_ENCODING, None
    return SUCCESS, k


def sk_to_pk(sk: int):
    return g1_mul(G1_GEN, sk)


def sign(sk: int, msg: bytes, dst: bytes = DST_POP):
    return g2_mul(hash_to_g2(msg, dst), sk)


def interop_secret_key(index: int) -> int:
    """interop/src/lib.rs:65-76: LE-int(SHA-256(hash_tree_root(u64 index))) mod r."""
    root = index.to_bytes(8, "little") + bytes(24)
    h = hashlib.sha256(root).digest()
    return int.from_bytes(h, "little") % R


def pk_validate(pk) -> int:
    """blst PublicKey::validate (public_key.rs:27)."""
    if pk is None:
        return PK_IS_INFINITY
    if not g1_in_group(pk):
        return POINT_NOT_IN_GROUP
    return SUCCESS


def public_key_from_bytes(data: bytes):
    """PublicKey: TryFrom<PublicKeyBytes> (public_key.rs:16-31) -> (status, pk)."""
    st, pk = g1_decompress(data)
    if st != SUCCESS:
        return st, None
    st = pk_validate(pk)
    return (st, pk) if st == SUCCESS else (st, None)


def signature_from_bytes(data: bytes):
    """Signature: TryFrom<SignatureBytes> (signature.rs:36-45): on-curve only."""
    return g2_decompress(data)


def aggregate_public_keys(pks):
    """PublicKey::aggregate_nonempty (public_key.rs:34-40) -> (status, pk)."""
    pks = list(pks)
    if not pks:
        return AGGR_TYPE_MISMATCH, None
    acc = None
    for pk in pks:
        acc = g1_add(acc, pk)
    return SUCCESS, acc


def aggregate_signatures(sigs):
    acc = None
    for s in sigs:
        acc = g2_add(acc, s)
    return acc


def _aggregate_verify_1(sig, msg, pk, sig_groupcheck: bool, dst: bytes) -> bool:
    """blst aggregate_verify with one (pk, msg): e(pk, H(m)) == e(g1, sig)."""
    if pk is None:  # PAIRING_Aggregate_PK_in_G1 rejects infinite PK
        return False
    if sig_groupcheck and sig is not None and not g2_in_group(sig):
        return False
    f = miller_loop(pk, hash_to_g2(msg, dst))
    if sig is not None:
        f = f12_mul(f, miller_loop(g1_neg(G1_GEN), sig))
    return f12_is_one(final_exp(f))


def verify(sig, msg: bytes, pk, dst: bytes = DST_POP) -> bool:
    """Signature::verify (signature.rs:47-60): sig_groupcheck = true, pk_validate = false."""
    return _aggregate_verify_1(sig, msg, pk, True, dst)


def fast_aggregate_verify(sig, msg: bytes, pks, dst: bytes = DST_POP) -> bool:
    """Signature::fast_aggregate_verify (signature.rs:77-93)."""
    st, agg = aggregate_public_keys(pks)
    if st != SUCCESS:
        return False
    return _aggregate_verify_1(sig, msg, agg, True, dst)


def multi_verify(msgs, sigs, pks, rands, dst: bytes = DST_POP) -> bool:
    """Signature::multi_verify (signature.rs:95-129) with caller-fixed 64-bit scalars.

    blst verify_multiple_aggregate_signatures(pks_validate=false, sigs_groupcheck=false,
    rand_bits=64): prod_i e(r_i pk_i, H(m_i)) * e(-sum r_i sig_i, g1) == 1.
    """
    n = len(pks)
    if n == 0 or len(msgs) != n or len(sigs) != n or len(rands) != n:
        return False
    f = f12_one()
    s_acc = None
    for m, s, pk, r in zip(msgs, sigs, pks, rands):
        r &= (1 << 64) - 1
        if pk is None:
            return False
        if s is not None:  # infinite signatures are skipped in the G2 sum
            s_acc = g2_add(s_acc, g2_mul(s, r))
        f = f12_mul(f, miller_loop(g1_mul(pk, r), hash_to_g2(m, dst)))
    if s_acc is not None:
        f = f12_mul(f, miller_loop(g1_neg(G1_GEN), s_acc))
    return f12_is_one(final_exp(f))
