"""CPU: the independent C oracle (oracle/bls_ref.c -- 64-bit limbs, textbook final
exponentiation; also bench.py's CPU baseline) against the committed golden fixtures
(pinned by the reference's KATs and RFC 9380 vectors) and against the Python oracle."""
import ctypes
import json
import os
import subprocess

import pytest

from oracle import bls12_381 as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
MONT = 1 << 384
RINV = pow(MONT, -1, O.P)


def gold(name):
    with open(os.path.join(GOLD, name + ".json")) as fh:
        return json.load(fh)


@pytest.fixture(scope="module")
def C():
    subprocess.check_call(["make", "-C", os.path.join(ROOT, "oracle"), "-s"])
    L = ctypes.CDLL(os.path.join(ROOT, "oracle", "_build", "libbls_ref.so"))
    L.ref_multi_verify.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p,
                                   ctypes.POINTER(ctypes.c_uint64), ctypes.c_size_t, ctypes.c_int]
    L.ref_verify.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p]
    L.ref_hash_to_g2.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p]
    L.ref_sign.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p]
    return L


def fp_b(x):
    return (x * MONT % O.P).to_bytes(48, "little")


def g1_b(p):
    return bytes(96) if p is None else fp_b(p[0]) + fp_b(p[1])


def g2_b(p):
    return bytes(192) if p is None else fp_b(p[0][0]) + fp_b(p[0][1]) + fp_b(p[1][0]) + fp_b(p[1][1])


def g2_of(b):
    v = [int.from_bytes(b[48 * k:48 * k + 48], "little") * RINV % O.P for k in range(4)]
    return None if not any(b) else ((v[0], v[1]), (v[2], v[3]))


def test_hash_to_g2_vectors(C):
    for c in gold("hash_to_g2")["cases"]:
        m, d = bytes.fromhex(c["msg"]), bytes.fromhex(c["dst"])
        out = ctypes.create_string_buffer(192)
        C.ref_hash_to_g2(m, len(m), d, len(d), out)
        v = [int.from_bytes(out.raw[48 * k:48 * k + 48], "little") * RINV % O.P for k in range(4)]
        assert ["%096x" % x for x in v] == c["x"] + c["y"]


def test_sign_and_keys(C):
    for c in gold("sign")["cases"]:
        out = ctypes.create_string_buffer(192)
        m = bytes.fromhex(c["msg"])
        C.ref_sign(bytes.fromhex(c["sk"]), m, len(m), out)
        assert O.g2_compress(g2_of(out.raw)).hex() == c["sig"]
    for c in gold("keys")["interop"]:
        out = ctypes.create_string_buffer(96)
        C.ref_sk_to_pk(bytes.fromhex(c["sk"]), out)
        x = int.from_bytes(out.raw[:48], "little") * RINV % O.P
        y = int.from_bytes(out.raw[48:], "little") * RINV % O.P
        assert O.g1_compress((x, y)).hex() == c["pk"]


def test_verify_fixtures(C):
    for c in gold("verify")["cases"]:
        sig = O.g2_decompress(bytes.fromhex(c["sig"]))[1]
        pk = O.g1_decompress(bytes.fromhex(c["pk"]))[1]
        m = bytes.fromhex(c["msg"])
        assert bool(C.ref_verify(g2_b(sig), m, len(m), g1_b(pk))) == c["expect"], c["note"]


@pytest.mark.parametrize("threads", [1, 3])
def test_multi_verify_fixtures(C, threads):
    for c in gold("multi_verify")["cases"]:
        n = len(c["msgs"])
        sigs = b"".join(g2_b(O.g2_decompress(bytes.fromhex(h))[1]) for h in c["sigs"])
        pks = b"".join(g1_b(O.g1_decompress(bytes.fromhex(h))[1]) for h in c["pks"])
        rands = (ctypes.c_uint64 * n)(*[int(r) for r in c["rands"]])
        msgs = b"".join(bytes.fromhex(h) for h in c["msgs"])
        assert bool(C.ref_multi_verify(msgs, sigs, pks, rands, n, threads)) == c["expect"], c["note"]


def test_baseline_driver_accepts_its_batch(C):
    exe = os.path.join(ROOT, "oracle", "_build", "bls_ref_bench")
    rec = json.loads(subprocess.check_output([exe, "24", "2"], text=True).strip())
    assert rec["ok"] == 1 and rec["n"] == 24 and rec["sets_per_s"] > 0


def test_fast_build_equals_textbook_build(C):
    """The CPU baseline's build (-DBLS_REF_FAST: Karatsuba Fp2/Fp6/Fp12, complex squarings,
    windowed exponentiations) computes the same field elements as the textbook checker:
    identical hash_to_G2 points, identical Miller partial bytes and the same verdicts on the
    golden multi_verify cases and on a signed 24-set batch (valid and corrupted)."""
    Fb = ctypes.CDLL(os.path.join(ROOT, "oracle", "_build", "libbls_ref_fast.so"))
    for L in (C, Fb):
        L.ref_multi_verify.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p,
                                       ctypes.POINTER(ctypes.c_uint64), ctypes.c_size_t, ctypes.c_int]
        L.ref_multi_verify_partial.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p,
                                               ctypes.POINTER(ctypes.c_uint64), ctypes.c_size_t, ctypes.c_char_p]
        L.ref_hash_to_g2.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t,
                                     ctypes.c_char_p]
        L.ref_sign.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p]
        L.ref_sk_to_pk.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
    for c in gold("hash_to_g2")["cases"]:
        m, d = bytes.fromhex(c["msg"]), bytes.fromhex(c["dst"])
        a, b = ctypes.create_string_buffer(192), ctypes.create_string_buffer(192)
        C.ref_hash_to_g2(m, len(m), d, len(d), a)
        Fb.ref_hash_to_g2(m, len(m), d, len(d), b)
        assert a.raw == b.raw
    for c in gold("multi_verify")["cases"]:
        n = len(c["msgs"])
        sigs = b"".join(g2_b(O.g2_decompress(bytes.fromhex(h))[1]) for h in c["sigs"])
        pks = b"".join(g1_b(O.g1_decompress(bytes.fromhex(h))[1]) for h in c["pks"])
        rands = (ctypes.c_uint64 * n)(*[int(r) for r in c["rands"]])
        msgs = b"".join(bytes.fromhex(h) for h in c["msgs"])
        assert bool(Fb.ref_multi_verify(msgs, sigs, pks, rands, n, 2)) == c["expect"], c["note"]
    n = 24
    import hashlib
    sks = [hashlib.sha256(b"fast%d" % i).digest() for i in range(n)]
    sks = [bytes([s[0] & 0x3F]) + s[1:] for s in sks]
    msgs = [hashlib.sha256(b"fm%d" % i).digest() for i in range(n)]
    pks, sigs = b"", b""
    for sk, m in zip(sks, msgs):
        p, s = ctypes.create_string_buffer(96), ctypes.create_string_buffer(192)
        C.ref_sk_to_pk(sk, p)
        C.ref_sign(sk, m, 32, s)
        pks += p.raw
        sigs += s.raw
    rands = (ctypes.c_uint64 * n)(*[(0x9E3779B97F4A7C15 * (i + 1)) % (1 << 64) or 1 for i in range(n)])
    mb = b"".join(msgs)
    pa, pb = ctypes.create_string_buffer(576), ctypes.create_string_buffer(576)
    assert C.ref_multi_verify_partial(mb, sigs, pks, rands, n, pa) == 0
    assert Fb.ref_multi_verify_partial(mb, sigs, pks, rands, n, pb) == 0
    assert pa.raw == pb.raw
    assert C.ref_multi_verify(mb, sigs, pks, rands, n, 2) == 1 and Fb.ref_multi_verify(mb, sigs, pks, rands, n, 2) == 1
    bad = sigs[:192 * 5] + sigs[192 * 6:192 * 7] + sigs[192 * 6:]
    assert C.ref_multi_verify(mb, bad, pks, rands, n, 2) == 0 and Fb.ref_multi_verify(mb, bad, pks, rands, n, 2) == 0
