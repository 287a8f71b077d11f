"""CPU: pin the oracle (oracle/bls12_381.py) against the reference's own KATs and the
committed golden vectors, plus algebraic self-checks."""
import json
import os
import random

import pytest

from oracle import bls12_381 as O

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def gold(name):
    with open(os.path.join(GOLD, name + ".json")) as fh:
        return json.load(fh)


def test_curve_order_matches_reference():  # interop/src/lib.rs:105-114
    assert str(O.R) == "52435875175126190479447740508185965837690552500527637822603658699938581184513"


def test_parameters():
    assert pow(3, O.P - 1, O.P) == 1 and pow(5, O.R - 1, O.R) == 1  # Fermat witnesses
    assert (O.P ** 4 - O.P ** 2 + 1) % O.R == 0
    assert O.g1_on_curve(O.G1_GEN) and O.g2_on_curve(O.G2_GEN)
    assert O.g1_mul(O.G1_GEN, O.R) is None and O.g2_mul(O.G2_GEN, O.R) is None


def test_interop_keygen_kats():  # interop/src/lib.rs:119-178
    for c in gold("keys")["interop"]:
        assert O.interop_secret_key(c["index"]) == int(c["sk"], 16)
        assert O.g1_compress(O.sk_to_pk(int(c["sk"], 16))).hex() == c["pk"]


def test_eip2335_pubkey():  # eip_2335/src/lib.rs:505,552
    k = gold("keys")["eip2335"]
    assert O.g1_compress(O.sk_to_pk(int(k["sk"], 16))).hex() == k["pk"]


def test_rfc9380_hash_to_g2_vectors():
    for c in gold("hash_to_g2")["cases"]:
        (x0, x1), (y0, y1) = O.hash_to_g2(bytes.fromhex(c["msg"]), bytes.fromhex(c["dst"]))
        assert ["%096x" % v for v in (x0, x1, y0, y1)] == c["x"] + c["y"]


def test_sign_vectors():
    for c in gold("sign")["cases"]:
        assert O.g2_compress(O.sign(int(c["sk"], 16), bytes.fromhex(c["msg"]))).hex() == c["sig"]


def test_isogeny_lands_on_e2_and_is_homomorphic():
    rng = random.Random(3)

    def rand_e2p():
        while True:
            x = (rng.randrange(O.P), rng.randrange(O.P))
            gx = O.f2_add(O.f2_add(O.f2_mul(O.f2_sqr(x), x), O.f2_mul(O.SSWU_A, x)), O.SSWU_B)
            y = O.f2_sqrt(gx)
            if y:
                return (x, y)

    a, b = rand_e2p(), rand_e2p()
    lam = O.f2_mul(O.f2_sub(b[1], a[1]), O.f2_inv(O.f2_sub(b[0], a[0])))
    x3 = O.f2_sub(O.f2_sub(O.f2_sqr(lam), a[0]), b[0])
    s = (x3, O.f2_sub(O.f2_mul(lam, O.f2_sub(a[0], x3)), a[1]))
    assert O.g2_on_curve(O.iso_map_g2(a))
    assert O.iso_map_g2(s) == O.g2_add(O.iso_map_g2(a), O.iso_map_g2(b))


def test_h_eff_equals_budroni_pintore():
    q = O.iso_map_g2(O.map_to_curve_sswu((5, 7)))
    assert O.clear_cofactor_g2(q) == O.clear_cofactor_g2_bp(q)


def test_pairing_bilinear_nondegenerate():
    e = O.pairing(O.G1_GEN, O.G2_GEN)
    assert not O.f12_is_one(e)
    assert O.f12_eq(O.pairing(O.g1_mul(O.G1_GEN, 6), O.g2_mul(O.G2_GEN, 7)), O.f12_pow(e, 42))


def test_g1_decode_fixture_statuses():
    for c in gold("g1_decode")["cases"]:
        st, p = O.g1_decompress(bytes.fromhex(c["in"]))
        assert st == c["status"]
        assert O.public_key_from_bytes(bytes.fromhex(c["in"]))[0] == c["validate_status"]


@pytest.mark.slow
def test_verdict_fixtures_replay():
    for c in gold("verify")["cases"]:
        sig = O.g2_decompress(bytes.fromhex(c["sig"]))[1]
        pk = O.g1_decompress(bytes.fromhex(c["pk"]))[1]
        assert O.verify(sig, bytes.fromhex(c["msg"]), pk) == c["expect"]


def test_trusted_setup_g2_points_in_group():
    raw = open(os.path.join(GOLD, "trusted_setup.bin"), "rb").read()
    n1 = int.from_bytes(raw[0:4], "little")
    n2 = int.from_bytes(raw[4:8], "little")
    assert (n1, n2) == (4096, 65)
    g2 = raw[8 + 48 * n1:]
    st, p = O.g2_decompress(g2[:96])
    assert st == 0 and p == O.G2_GEN  # line 4099 = [1]G2
    st, p = O.g2_decompress(g2[96:192])
    assert st == 0 and O.g2_in_group(p) and O.g2_compress(p) == g2[96:192]
