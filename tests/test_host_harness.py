"""CPU: the engine's own device arithmetic (grandine_amd/csrc/*.h), compiled for the host
by tests/native/host_harness.cpp, against the golden fixtures and the oracle."""
import ctypes
import json
import os
import subprocess

import pytest

from oracle import bls12_381 as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
SO = os.path.join(ROOT, "tests", "native", "_build", "libhost_harness.so")
# GBLS_HARNESS_SAN=1 (tests/test_host_sanitizers.py): an ASan + UBSan build of the same harness,
# loaded by a child interpreter that preloads libasan
SAN = os.environ.get("GBLS_HARNESS_SAN") == "1"
if SAN:
    SO = os.path.join(ROOT, "tests", "native", "_build", "libhost_harness_san.so")
RINV = pow(1 << 384, -1, O.P)


def gold(name):
    with open(os.path.join(GOLD, name + ".json")) as fh:
        return json.load(fh)


@pytest.fixture(scope="module")
def H():
    src = os.path.join(ROOT, "tests", "native", "host_harness.cpp")
    os.makedirs(os.path.dirname(SO), exist_ok=True)
    # GBLS_HARNESS_DEFS: extra -D flags, to check an experiment build's arithmetic (e.g.
    # -DGBLS_POW_ENGINE) with the same tests
    defs = os.environ.get("GBLS_HARNESS_DEFS", "").split()
    opt = (["-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined", "-fno-sanitize-recover=all"]
           if SAN else ["-O2"])
    # GBLS_R28_CHECK: the radix-2^28 layer's limb contracts checked on every operation (abort)
    subprocess.check_call(["g++"] + opt + ["-std=c++17", "-shared", "-fPIC", "-D__HIP_PLATFORM_AMD__",
                           "-DGBLS_R28_CHECK", "-I/opt/rocm/include"] + defs + ["-o", SO, src])
    L = ctypes.CDLL(SO)
    L.h_multi_verify.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p,
                                 ctypes.POINTER(ctypes.c_uint64), ctypes.c_uint32]
    return L


def fp_b(x):
    return (x * (1 << 384) % O.P).to_bytes(48, "little")


def g1_b(p):
    return bytes(96) if p is None else fp_b(p[0]) + fp_b(p[1])


def g2_b(p):
    return bytes(192) if p is None else fp_b(p[0][0]) + fp_b(p[0][1]) + fp_b(p[1][0]) + fp_b(p[1][1])


def test_fp_mul_random(H):
    import random
    rng = random.Random(1)
    for _ in range(200):
        a, b = rng.randrange(O.P), rng.randrange(O.P)
        out = ctypes.create_string_buffer(48)
        H.h_fp_mul(a.to_bytes(48, "little"), b.to_bytes(48, "little"), out)
        assert int.from_bytes(out.raw, "little") == a * b * pow(1 << 384, -1, O.P) % O.P


def test_fp_inv(H):
    """fp_inv (the safegcd of bls_inv.h since r04) times its input is 1."""
    import random
    rng = random.Random(2)
    for a in [1, 2, O.P - 1, O.P - 2] + [rng.randrange(1, O.P) for _ in range(100)]:
        out = ctypes.create_string_buffer(48)
        assert H.h_fp_inv_check(a.to_bytes(48, "little"), out) == 1
        # Montgomery: input aR -> output a^-1 R
        want = pow(a * RINV % O.P, -1, O.P) * (1 << 384) % O.P
        assert int.from_bytes(out.raw, "little") == want


def test_fp_inv_var_safegcd(H):
    """bls_inv.h (safegcd, 30-divstep batches, variable time) against Python's modular
    inverse: edge values, values just below p, powers of two, and random values."""
    import random
    rng = random.Random(21)
    vals = [0, 1, 2, 3, O.P - 1, O.P - 2, (O.P - 1) // 2, (O.P + 1) // 2, 1 << 380, (1 << 381) % O.P]
    vals += [(1 << k) % O.P for k in range(0, 381, 29)]
    vals += [rng.randrange(1, O.P) for _ in range(3000)]
    vals += [rng.randrange(1, 1 << rng.randrange(1, 381)) for _ in range(300)]
    for a in vals:
        out = ctypes.create_string_buffer(48)
        H.h_fp_inv_var(a.to_bytes(48, "little"), out)
        got = int.from_bytes(out.raw, "little")
        want = 0 if a == 0 else pow(a * RINV % O.P, -1, O.P) * (1 << 384) % O.P
        assert got == want, hex(a)


def test_wave12_product_matches_tower_product(H):
    """The wave-cooperative Fp12 product (generated linear maps, 54 lanes) equals the
    tower Karatsuba product, including on extreme coefficients (0, 1, p-1)."""
    import random
    rng = random.Random(3)
    specials = [0, 1, O.P - 1]
    for t in range(40):
        if t < 3:
            av = [specials[t]] * 12
            bv = [specials[(t + 1) % 3]] * 12
        else:
            av = [rng.choice(specials) if rng.random() < 0.2 else rng.randrange(O.P) for _ in range(12)]
            bv = [rng.choice(specials) if rng.random() < 0.2 else rng.randrange(O.P) for _ in range(12)]
        a = b"".join(x.to_bytes(48, "little") for x in av)
        b = b"".join(x.to_bytes(48, "little") for x in bv)
        o1 = ctypes.create_string_buffer(576)
        o2 = ctypes.create_string_buffer(576)
        H.h_fp12_mul_w12(a, b, o1)
        H.h_fp12_mul_ref(a, b, o2)
        assert o1.raw == o2.raw


def test_g1_windowed_scalar_product(H):
    """g1_mul_u64_w3 (k_mv_g1mul_lane: signed 3-bit windows over {P, 2P, 3P, 4P}) equals
    the double-and-add mul_u64 on edge scalars (0, small, every digit value, top bit,
    all ones) and random ones, and maps the point at infinity to infinity."""
    import random
    rng = random.Random(5)
    H.h_g1_mul_w3_check.argtypes = [ctypes.c_char_p, ctypes.c_uint64]
    pts = [g1_b(O.sk_to_pk(sk)) for sk in (1, 7, 0x1234567890ABCDEF)] + [bytes(96)]
    ks = [0, 1, 2, 3, 4, 5, 6, 7, 8, 0o4444, 0o3333, 0o77777, 1 << 63, (1 << 63) - 1, (1 << 64) - 1,
          0x9E3779B97F4A7C15, 0x4924924924924924] + [rng.getrandbits(64) for _ in range(40)]
    for p in pts:
        for k in ks:
            assert H.h_g1_mul_w3_check(p, k) == 1, (p.hex()[:16], k)


def test_g1_decode_fixtures(H):
    for c in gold("g1_decode")["cases"]:
        out = ctypes.create_string_buffer(96)
        assert H.h_g1_decompress(bytes.fromhex(c["in"]), 0, out) == c["status"]
        assert H.h_g1_decompress(bytes.fromhex(c["in"]), 1, out) == c["validate_status"]
        if c["validate_status"] == 0:
            enc = ctypes.create_string_buffer(48)
            H.h_g1_compress(out, enc)
            assert enc.raw.hex() == c["out"]


def test_g2_decode_fixtures(H):
    for c in gold("g2_decode")["cases"]:
        out = ctypes.create_string_buffer(192)
        assert H.h_g2_decompress(bytes.fromhex(c["in"]), out) == c["status"]
        if c["status"] == 0:
            enc = ctypes.create_string_buffer(96)
            H.h_g2_compress(out, enc)
            assert enc.raw.hex() == c["out"]
            assert bool(H.h_g2_in_group(out)) == c["in_group"]


def test_hash_to_g2_fixtures(H):
    for c in gold("hash_to_g2")["cases"]:
        m, d = bytes.fromhex(c["msg"]), bytes.fromhex(c["dst"])
        out = ctypes.create_string_buffer(192)
        H.h_hash_to_g2(m, len(m), d, len(d), out)
        v = [int.from_bytes(out.raw[48 * k:48 * k + 48], "little") * RINV % O.P for k in range(4)]
        assert ["%096x" % x for x in v] == c["x"] + c["y"]


def test_verify_fixtures(H):
    for c in gold("verify")["cases"]:
        sig = O.g2_decompress(bytes.fromhex(c["sig"]))[1]
        pk = O.g1_decompress(bytes.fromhex(c["pk"]))[1]
        m = bytes.fromhex(c["msg"])
        assert (H.h_verify(g2_b(sig), m, len(m), g1_b(pk)) == 0) == c["expect"], c["note"]


def test_multi_verify_fixtures(H):
    for c in gold("multi_verify")["cases"]:
        n = len(c["msgs"])
        sigs = b"".join(g2_b(O.g2_decompress(bytes.fromhex(h))[1]) for h in c["sigs"])
        pks = b"".join(g1_b(O.g1_decompress(bytes.fromhex(h))[1]) for h in c["pks"])
        rands = (ctypes.c_uint64 * n)(*[int(r) for r in c["rands"]])
        msgs = b"".join(bytes.fromhex(h) for h in c["msgs"])
        assert (H.h_multi_verify(msgs, sigs, pks, rands, n) == 0) == c["expect"], c["note"]


def test_inversion_free_final_verdict(H):
    """k_final_verdict's test "Psi(f^(p^2+1)) has zero w-half" equals the textbook
    "final_exp(f) == 1": on a valid batch's Miller product (true), on that product times
    Fp6 elements (killed by the p^6 - 1 of the final exponentiation: still true), and on
    products times elements outside Fp6 (false)."""
    import random
    rng = random.Random(11)
    C = ctypes.CDLL(os.path.join(ROOT, "oracle", "_build", "libbls_ref.so"))
    C.ref_multi_verify_partial.argtypes = [ctypes.c_char_p] * 3 + [ctypes.POINTER(ctypes.c_uint64), ctypes.c_size_t,
                                                                   ctypes.c_char_p]
    cases = gold("multi_verify")["cases"]
    c = next(x for x in cases if x["expect"] and len(x["msgs"]) >= 6)
    msgs = b"".join(bytes.fromhex(h) for h in c["msgs"])
    sigs = b"".join(g2_b(O.g2_decompress(bytes.fromhex(h))[1]) for h in c["sigs"])
    pks = b"".join(g1_b(O.g1_decompress(bytes.fromhex(h))[1]) for h in c["pks"])
    n = len(c["msgs"])
    part = ctypes.create_string_buffer(576)
    assert C.ref_multi_verify_partial(msgs, sigs, pks, (ctypes.c_uint64 * n)(*[int(r) for r in c["rands"]]), n,
                                      part) == 0
    f = part.raw
    assert H.h_final_exp_is_one(f) == 1 and H.h_w12_verdict(f) == 1
    out = ctypes.create_string_buffer(576)
    for trial in range(6):
        coefs = [rng.randrange(O.P) for _ in range(12)]
        if trial < 3:
            coefs[6:] = [0] * 6  # an Fp6 element
        H.h_fp12_mul(f, b"".join(fp_b(x) for x in coefs), out)
        want = H.h_final_exp_is_one(out.raw)
        assert want == (trial < 3)
        assert H.h_w12_verdict(out.raw) == want
    assert H.h_w12_verdict(bytes(576)) == 0


def test_radix28_field_layer(H):
    """bls_field28.h (the next field layer) against Python big integers, through
    the engine form: conversions, product, dual product, subtraction, Fp2 product/square."""
    import random
    rng = random.Random(28)
    H.h_r28_op.argtypes = [ctypes.c_int] + [ctypes.c_char_p] * 4 + [ctypes.c_void_p] * 2
    R = 1 << 384
    m = lambda x: (x * R % O.P).to_bytes(48, "little")  # engine (Montgomery-384) form
    edge = [0, 1, 2, O.P - 1, O.P - 2, (1 << 380), O.P // 2]
    vals = edge + [rng.randrange(O.P) for _ in range(120)]
    for i in range(len(vals)):
        a, b, c, d = vals[i], vals[-1 - i], rng.choice(vals), rng.choice(vals)
        r, r2 = ctypes.create_string_buffer(48), ctypes.create_string_buffer(48)

        def run(op):
            ret = H.h_r28_op(op, m(a), m(b), m(c), m(d), r, r2)
            got = int.from_bytes(r.raw, "little") * RINV % O.P
            got2 = int.from_bytes(r2.raw, "little") * RINV % O.P
            assert int.from_bytes(r.raw, "little") < O.P  # canonical engine form
            return ret, got, got2
        assert run(0)[1] == a
        assert run(1)[1] == a * b % O.P
        assert run(2)[1] == (a * b + c * d) % O.P
        assert run(3)[1] == (a - b) % O.P
        _, g0, g1 = run(4)
        assert (g0, g1) == ((a * c - b * d) % O.P, (a * d + b * c) % O.P)
        _, g0, g1 = run(5)
        assert (g0, g1) == ((a * a - b * b) % O.P, 2 * a * b % O.P)
        assert run(6)[0] == (a == b)
    r, r2 = ctypes.create_string_buffer(48), ctypes.create_string_buffer(48)
    assert H.h_r28_op(6, m(5), m(5), m(0), m(0), r, r2) == 1


def test_radix28_sparse_miller_products(H):
    """bls_field28.h's sparse Miller products (the r28 k_ml_group path) equal the engine's
    (bls_pairing.h) on random operands, through 40-step dense x sparse chains that rotate over
    every form (Karatsuba, Karatsuba with the LDS stash, and the k_ml_group28 lazy forms with one
    reduction per output coordinate, in place, with and without parked outputs), and the lazy
    sparse x sparse product; sp_from_engine differs from line_eval_s by one scalar shared by all
    coefficients."""
    H.h_r28_tower_check.argtypes = [ctypes.c_uint64, ctypes.c_int, ctypes.c_int]
    assert H.h_r28_tower_check(7, 30, 40) == 0


def test_radix28_miller_line_steps(H):
    """The radix-2^28 line steps of k_lines_lane28 (bls_curve28.h line_dbl28 / line_add28, the
    store-as-known order) equal the engine's line_dbl / line_add_aff (bls_pairing.h) at every
    one of the 68 events from random points, coefficient by coefficient, and the running point
    T at the end; the repacked storage form reads back as the same value."""
    H.h_r28_lines_check.argtypes = [ctypes.c_uint64]
    for seed in range(1, 9):
        assert H.h_r28_lines_check(seed) == 0, seed


def test_radix28_cofactor_clearing(H):
    """The lane-regime cofactor clearing in the radix-2^28 layer (bls_curve28.h: the engine's
    Jacobian templates over r28::fe2, psi / psi^2 with radix-2^28 constants) equals the
    engine's clear_cofactor_g2 on Q0 + Q1 of seeded messages."""
    H.h_r28_clear_check.argtypes = [ctypes.c_char_p, ctypes.c_uint32]
    for i in range(4):
        m = b"r28-clear/%d" % i
        assert H.h_r28_clear_check(m, len(m)) == 1, i


def test_radix28_g1_scalar_multiplication(H):
    """The lane-regime r_i pk_i in the radix-2^28 layer (bls_curve28.h g1_mul_u64_w3_28 over
    r28::fe with the dedicated square, g1s_from_jac28) equals the engine's g1_mul_u64_w3 +
    g1s_from_jac as a point (the scaled form (X Z, Y, Z^3) compared through cross products)."""
    H.h_r28_g1mul_check.argtypes = [ctypes.c_uint64, ctypes.c_int]
    for seed in (1, 77, 0xDEADBEEF):
        assert H.h_r28_g1mul_check(seed, 6) == 0, seed



def test_radix28_g2_subgroup_check(H):
    """bls_curve28.h g2_in_group28 (k_g2_check28: psi(P) == [x]P with lazy doublings and mixed
    additions of the affine base) equals the engine's g2_in_group: true for cleared hash points,
    false for the uncleared map outputs (on E2, outside G2)."""
    H.h_r28_g2check.argtypes = [ctypes.c_char_p, ctypes.c_uint32]
    for i in range(4):
        m = b"r28-g2check/%d" % i
        assert H.h_r28_g2check(m, len(m)) == 1, i


def test_radix28_lazy_doubling(H):
    """bls_curve28.h jac_dbl28 / jac_add28 / jac_add_aff28 (lazy combinations, weak reductions
    only where an output or a square's operand needs one) equal bls_curve.h's jac_dbl / jac_add /
    jac_add_aff over the reduced f_ operations, for G2 (r28::fe2) and G1 (r28::fe) coordinates,
    from inputs at the top of their contract (< 2.03 p) through 70 chained doublings with an
    addition of a Jacobian or an affine point after two of every three;
    the harness is built with GBLS_R28_CHECK, so every combination's limb contract is checked."""
    H.h_r28_dbl_check.argtypes = [ctypes.c_uint64, ctypes.c_int]
    for seed in (1, 2, 3, 0xdeadbeef):
        assert H.h_r28_dbl_check(seed, 70) == 0, seed
