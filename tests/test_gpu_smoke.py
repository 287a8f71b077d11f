"""First on-device parity checks against the oracle (small sizes)."""
import ctypes

import pytest

from oracle import bls12_381 as O

pytestmark = pytest.mark.gpu

RINV = pow(1 << 384, -1, O.P)


def _fp(b):
    return int.from_bytes(b, "little") * RINV % O.P


def _g2_of(b):
    if not any(b):
        return None
    return ((_fp(b[:48]), _fp(b[48:96])), (_fp(b[96:144]), _fp(b[144:])))


def test_hash_to_g2_rfc_vector():
    from grandine_amd import _lib as G
    L = G.lib()
    dst = b"QUUX-V01-CS02-with-BLS12381G2_XMD:SHA-256_SSWU_RO_"
    msgs = [b"", b"abc"]
    data = b"".join(msgs)
    off = G.u32_array([0, 0, 3])
    out = ctypes.create_string_buffer(192 * 2)
    G.check(L.gbls_hash_to_g2(data or b"\0", off, 2, dst, len(dst), out), "h2c")
    for i, m in enumerate(msgs):
        assert _g2_of(out.raw[192 * i:192 * (i + 1)]) == O.hash_to_g2(m, dst)


def test_sign_and_multi_verify_small():
    from grandine_amd import _lib as G
    L = G.lib()
    n = 5
    sks = [O.interop_secret_key(i) for i in range(n)]
    msgs = b"".join(bytes([i + 1]) * 32 for i in range(n))
    skb = b"".join(k.to_bytes(32, "big") for k in sks)
    pks = ctypes.create_string_buffer(96 * n)
    sigs = ctypes.create_string_buffer(192 * n)
    G.check(L.gbls_sk_to_pk(skb, n, pks), "sk_to_pk")
    G.check(L.gbls_sign(skb, msgs, G.u32_array(range(0, 32 * n + 1, 32)), n, sigs), "sign")
    for i in range(n):
        assert _g2_of(sigs.raw[192 * i:192 * (i + 1)]) == O.sign(sks[i], msgs[32 * i:32 * i + 32])
    rands = G.u64_array([3 + 11 * i for i in range(n)])
    assert L.gbls_multi_verify(msgs, sigs, pks, rands, n) == G.SUCCESS
    bad = bytearray(msgs)
    bad[40] ^= 1
    assert L.gbls_multi_verify(bytes(bad), sigs, pks, rands, n) == G.VERIFY_FAIL
