"""On-device parity: every C-ABI entry point against the committed golden fixtures
(tests/golden, pinned to the reference's KATs and the oracle) and, at full batch sizes,
against size-independent properties.  Bit-exact for every byte / verdict.
"""

import ctypes
import hashlib
import json
import os

import pytest

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def gold(name):
    with open(os.path.join(GOLD, name + ".json")) as fh:
        return json.load(fh)


@pytest.fixture(scope="module")
def L():
    from grandine_amd import _lib as G
    return G.lib()


@pytest.fixture(scope="module")
def G():
    from grandine_amd import _lib as G
    return G


@pytest.fixture(scope="module")
def B():
    from grandine_amd import bls
    return bls


def _pk(B, hexstr):
    if hexstr == "c0" + "00" * 47:
        return B.PublicKey.default()
    st, raw = B.decompress_public_keys([bytes.fromhex(hexstr)], validate=False)[0]
    assert st == 0
    return B.PublicKey(raw)


def _sig(B, hexstr):
    return B.Signature.try_from(bytes.fromhex(hexstr))


# ------------------------------------------------------------------ keys / encodings
def test_interop_and_eip2335_keys(B):
    k = gold("keys")
    sks = [bytes.fromhex(c["sk"]) for c in k["interop"]] + [bytes.fromhex(k["eip2335"]["sk"])]
    want = [c["pk"] for c in k["interop"]] + [k["eip2335"]["pk"]]
    got = [p.to_bytes().hex() for p in B.public_keys_batch(sks)]
    assert got == want


def test_g1_decode_cases(L, G):
    cases = gold("g1_decode")["cases"]
    n = len(cases)
    inb = G.buf(b"".join(bytes.fromhex(c["in"]) for c in cases))
    for validate in (0, 1):
        out = ctypes.create_string_buffer(96 * n)
        st = G.i32_array(n)
        G.check(L.gbls_g1_decompress(inb, n, validate, out, st), "decompress")
        for i, c in enumerate(cases):
            assert st[i] == (c["validate_status"] if validate else c["status"]), (i, c)
        if not validate:
            ok = [i for i, c in enumerate(cases) if c["status"] == 0]
            enc = ctypes.create_string_buffer(48 * len(ok))
            pts = G.buf(b"".join(out.raw[96 * i:96 * i + 96] for i in ok))
            G.check(L.gbls_g1_compress(pts, len(ok), enc), "compress")
            for j, i in enumerate(ok):
                assert enc.raw[48 * j:48 * j + 48].hex() == cases[i]["out"]


def test_g2_decode_cases(L, G):
    cases = gold("g2_decode")["cases"]
    n = len(cases)
    out = ctypes.create_string_buffer(192 * n)
    st = G.i32_array(n)
    G.check(L.gbls_g2_decompress(G.buf(b"".join(bytes.fromhex(c["in"]) for c in cases)), n, out, st), "g2")
    ok = [i for i, c in enumerate(cases) if c["status"] == 0]
    for i, c in enumerate(cases):
        assert st[i] == c["status"], (i, c)
    pts = G.buf(b"".join(out.raw[192 * i:192 * i + 192] for i in ok))
    enc = ctypes.create_string_buffer(96 * len(ok))
    G.check(L.gbls_g2_compress(pts, len(ok), enc), "compress")
    grp = G.i32_array(len(ok))
    G.check(L.gbls_g2_validate(pts, len(ok), grp), "validate")
    for j, i in enumerate(ok):
        assert enc.raw[96 * j:96 * j + 96].hex() == cases[i]["out"]
        assert (grp[j] == 0) == cases[i]["in_group"], (i, cases[i])


def test_trusted_setup_points_decode_and_sum(L, G):
    """kzg_utils/src/trusted_setup.txt: all points decode, re-encode byte-identical,
    lie in their groups, and the 4096 G1 Lagrange points sum to the G1 generator."""
    raw = open(os.path.join(GOLD, "trusted_setup.bin"), "rb").read()
    n1 = int.from_bytes(raw[0:4], "little")
    n2 = int.from_bytes(raw[4:8], "little")
    g1 = raw[8:8 + 48 * n1]
    g2 = raw[8 + 48 * n1:8 + 48 * n1 + 96 * n2]
    out1 = ctypes.create_string_buffer(96 * n1)
    st1 = G.i32_array(n1)
    G.check(L.gbls_g1_decompress(G.buf(g1), n1, 1, out1, st1), "g1")
    assert all(st1[i] == 0 for i in range(n1))
    enc1 = ctypes.create_string_buffer(48 * n1)
    G.check(L.gbls_g1_compress(out1, n1, enc1), "c1")
    assert enc1.raw == g1
    agg = ctypes.create_string_buffer(96)
    assert L.gbls_g1_aggregate(out1, n1, agg) == 0
    enc = ctypes.create_string_buffer(48)
    G.check(L.gbls_g1_compress(agg, 1, enc), "c")
    assert enc.raw.hex() == ("97f1d3a73197d7942695638c4fa9ac0fc3688c4f9774b905a14e3a3f171bac586c55e83ff97a1aeffb3af00adb22c6bb")
    out2 = ctypes.create_string_buffer(192 * n2)
    st2 = G.i32_array(n2)
    G.check(L.gbls_g2_decompress(G.buf(g2), n2, out2, st2), "g2")
    assert all(st2[i] == 0 for i in range(n2))
    grp = G.i32_array(n2)
    G.check(L.gbls_g2_validate(out2, n2, grp), "v")
    assert all(grp[i] == 0 for i in range(n2))
    enc2 = ctypes.create_string_buffer(96 * n2)
    G.check(L.gbls_g2_compress(out2, n2, enc2), "c2")
    assert enc2.raw == g2


# ------------------------------------------------------------------ hash / sign
def test_hash_to_g2_vectors(L, G):
    from oracle import bls12_381 as O
    cases = gold("hash_to_g2")["cases"]
    for c in cases:
        msg = bytes.fromhex(c["msg"])
        dst = bytes.fromhex(c["dst"])
        out = ctypes.create_string_buffer(192)
        G.check(L.gbls_hash_to_g2(G.buf(msg), G.u32_array([0, len(msg)]), 1, dst, len(dst), out), "h2c")
        rinv = pow(1 << 384, -1, O.P)
        limbs = [int.from_bytes(out.raw[48 * k:48 * k + 48], "little") * rinv % O.P for k in range(4)]
        assert ["%096x" % v for v in limbs] == [c["x"][0], c["x"][1], c["y"][0], c["y"][1]]


def test_sign_vectors(B):
    cases = gold("sign")["cases"]
    sigs = B.sign_batch([bytes.fromhex(c["sk"]) for c in cases], [bytes.fromhex(c["msg"]) for c in cases])
    assert [s.to_bytes().hex() for s in sigs] == [c["sig"] for c in cases]


# ------------------------------------------------------------------ aggregation
def test_aggregate_cases(B):
    a = gold("aggregate")
    for c in a["g1"]:
        keys = [_pk(B, h) for h in c["pks"]]
        if c["status"] != 0:
            with pytest.raises(B.NoPublicKeysToAggregate):
                B.PublicKey.aggregate_nonempty(keys)
            continue
        assert B.PublicKey.aggregate_nonempty(keys).to_bytes().hex() == c["out"]
    for c in a["g2"]:
        sigs = [_sig(B, h) for h in c["sigs"]]
        acc = sigs[0]
        for s in sigs[1:]:
            acc = acc.aggregate(s)
        assert acc.to_bytes().hex() == c["out"]


def test_aggregate_segments_api(L, G, B):
    a = gold("aggregate")["g1"]
    keys, off = [], [0]
    for c in a:
        keys += [_pk(B, h).raw for h in c["pks"]]
        off.append(len(keys))
    n = len(a)
    out = ctypes.create_string_buffer(96 * n)
    st = G.i32_array(n)
    G.check(L.gbls_g1_aggregate_segments(G.buf(b"".join(keys)), G.u32_array(off), n, out, st), "seg")
    for i, c in enumerate(a):
        assert st[i] == c["status"]
        if c["status"] == 0:
            assert B.PublicKey(out.raw[96 * i:96 * i + 96]).to_bytes().hex() == c["out"]


def test_aggregate_segments_rows(L, G, B):
    """>= 128 segments take the row-per-segment kernel (k_aggregate_rows): the golden
    G1 / G2 aggregation cases repeated 64 times, and registry indices (out-of-range and
    empty segments included), against the golden outputs and the 256-lane form."""
    a = gold("aggregate")
    reps = 64
    keys, off, want = [], [0], []
    for _ in range(reps):
        for c in a["g1"]:
            keys += [_pk(B, h).raw for h in c["pks"]]
            off.append(len(keys))
            want.append(c)
    n = len(want)
    assert n >= 128
    out = ctypes.create_string_buffer(96 * n)
    st = G.i32_array(n)
    G.check(L.gbls_g1_aggregate_segments(G.buf(b"".join(keys)), G.u32_array(off), n, out, st), "rows g1")
    for i, c in enumerate(want):
        assert st[i] == c["status"]
        if c["status"] == 0:
            assert B.PublicKey(out.raw[96 * i:96 * i + 96]).to_bytes().hex() == c["out"]
    # G2
    sigs, off2, want2 = [], [0], []
    for _ in range(reps):
        for c in a["g2"]:
            sigs += [_sig(B, h).raw for h in c["sigs"]]
            off2.append(len(sigs))
            want2.append(c["out"])
    m = len(want2)
    assert m >= 128
    out2 = ctypes.create_string_buffer(192 * m)
    st2 = G.i32_array(m)
    G.check(L.gbls_g2_aggregate_segments(G.buf(b"".join(sigs)), G.u32_array(off2), m, out2, st2), "rows g2")
    for i, h in enumerate(want2):
        assert st2[i] == 0
        assert B.Signature(out2.raw[192 * i:192 * i + 192]).to_bytes().hex() == h
    # registry indices: row kernel vs the workgroup kernel (few segments) on the same data
    from grandine_amd import factory as F
    nreg = 4096
    _, comp = F.registry(nreg, seed=b"rows")
    assert not F.load_registry(comp).any()
    import numpy as np
    rng = np.random.default_rng(7)
    sizes = rng.integers(0, 40, size=300)
    sizes[5] = 0
    idx = rng.integers(0, nreg, size=int(sizes.sum()), dtype=np.uint32)
    offs = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint32)
    # out of range in segment 9 (sizes[9] > 0 checked below): past the registry's current size,
    # which earlier tests of the same process may have grown beyond nreg
    idx[int(offs[9])] = max(nreg, L.gbls_registry_size()) + 3
    assert sizes[9] > 0
    ns = len(sizes)
    o_rows = ctypes.create_string_buffer(96 * ns)
    s_rows = G.i32_array(ns)
    G.check(L.gbls_g1_aggregate_indexed(idx.ctypes.data_as(ctypes.c_void_p), offs.ctypes.data_as(ctypes.c_void_p),
                                        ns, o_rows, s_rows), "rows idx")
    for k in range(0, ns, 100):  # the same segments, 100 at a time: workgroup kernel
        cnt = min(100, ns - k)
        sub_off = (offs[k:k + cnt + 1] - offs[k]).astype(np.uint32)
        sub_idx = np.ascontiguousarray(idx[offs[k]:offs[k + cnt]])
        o_wg = ctypes.create_string_buffer(96 * cnt)
        s_wg = G.i32_array(cnt)
        G.check(L.gbls_g1_aggregate_indexed(sub_idx.ctypes.data_as(ctypes.c_void_p),
                                            sub_off.ctypes.data_as(ctypes.c_void_p), cnt, o_wg, s_wg), "wg idx")
        for j in range(cnt):
            assert s_rows[k + j] == s_wg[j], k + j
            assert o_rows.raw[96 * (k + j):96 * (k + j + 1)] == o_wg.raw[96 * j:96 * (j + 1)], k + j
    assert s_rows[5] == G.AGGR_TYPE_MISMATCH and s_rows[9] == G.BAD_ENCODING


# ------------------------------------------------------------------ verdicts
def test_verify_cases(B):
    for c in gold("verify")["cases"]:
        sig = _sig(B, c["sig"])
        assert sig.verify(bytes.fromhex(c["msg"]), _pk(B, c["pk"])) == c["expect"], c["note"]


def test_aggregate_verify_batch_matches_single(L, G, B):
    cases = gold("verify")["cases"]
    m = len(cases)
    msgs = [bytes.fromhex(c["msg"]) for c in cases]
    off = [0]
    for x in msgs:
        off.append(off[-1] + len(x))
    v = G.i32_array(m)
    G.check(L.gbls_aggregate_verify_batch(G.buf(b"".join(_sig(B, c["sig"]).raw for c in cases)), G.buf(b"".join(msgs)),
                                          G.u32_array(off), G.buf(b"".join(_pk(B, c["pk"]).raw for c in cases)), m, v),
            "batch")
    assert [v[i] == 0 for i in range(m)] == [c["expect"] for c in cases]


def test_fast_aggregate_verify_cases(B):
    for c in gold("fast_aggregate_verify")["cases"]:
        sig = _sig(B, c["sig"])
        keys = [_pk(B, h) for h in c["pks"]]
        assert sig.fast_aggregate_verify(bytes.fromhex(c["msg"]), keys) == c["expect"], c["note"]


def test_multi_verify_cases(B):
    for c in gold("multi_verify")["cases"]:
        msgs = [bytes.fromhex(h) for h in c["msgs"]]
        sigs = [_sig(B, h) for h in c["sigs"]]
        pks = [_pk(B, h) for h in c["pks"]]
        rands = [int(r) for r in c["rands"]]
        assert B.Signature.multi_verify(msgs, sigs, pks, rands) == c["expect"], c["note"]


def test_multi_verify_segments_independent_verdicts(L, G, B):
    cases = gold("multi_verify")["cases"]
    msgs, sigs, pks, rands, off = [], [], [], [], [0]
    for c in cases:
        msgs += [bytes.fromhex(h) for h in c["msgs"]]
        sigs += [_sig(B, h).raw for h in c["sigs"]]
        pks += [_pk(B, h).raw for h in c["pks"]]
        rands += [int(r) for r in c["rands"]]
        off.append(len(msgs))
    v = G.i32_array(len(cases))
    G.check(L.gbls_multi_verify_segments(G.buf(b"".join(msgs)), G.buf(b"".join(sigs)), G.buf(b"".join(pks)),
                                         G.u64_array(rands), len(msgs), G.u32_array(off), len(cases), v), "segs")
    assert [v[i] == 0 for i in range(len(cases))] == [c["expect"] for c in cases]


# ------------------------------------------------------------------ verifier mirror
def test_multi_verifier_finish(B):
    from grandine_amd import verifier as V
    k = gold("keys")["interop"]
    sks = [bytes.fromhex(c["sk"]) for c in k[:4]]
    msgs = [hashlib.sha256(b"mv%d" % i).digest() for i in range(4)]
    sigs = B.sign_batch(sks, msgs)
    pks = B.public_keys_batch(sks)
    mv = V.MultiVerifier()
    for m, s, p in zip(msgs, sigs, pks):
        mv.verify_singular(m, s.to_bytes(), B.CachedPublicKey(p.to_bytes()), V.SignatureKind.Block)
    mv.finish()
    mv.triples[1].message = msgs[2]
    with pytest.raises(V.SignatureInvalid):
        mv.finish()
    V.MultiVerifier().finish()  # verifier.rs:446-449


# ------------------------------------------------------------------ full-size properties
def _workload(B, n, seed=b"c2"):
    R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
    sks = [(int.from_bytes(hashlib.sha256(seed + b"sk%d" % i).digest(), "big") % R).to_bytes(32, "big")
           for i in range(n)]
    msgs = [hashlib.sha256(seed + b"m%d" % i).digest() for i in range(n)]
    return sks, msgs, B.sign_batch(sks, msgs), B.public_keys_batch(sks)


def test_c2_batch_4096_accept_and_reject(B):
    n = 4096
    sks, msgs, sigs, pks = _workload(B, n)
    rands = [(i * 0x9E3779B97F4A7C15 + 7) % (1 << 64) or 1 for i in range(n)]
    assert B.Signature.multi_verify(msgs, sigs, pks, rands)
    bad = list(sigs)
    bad[1234] = sigs[1235]
    assert not B.Signature.multi_verify(msgs, bad, pks, rands)
    badm = list(msgs)
    badm[4095] = hashlib.sha256(b"other").digest()
    assert not B.Signature.multi_verify(badm, sigs, pks, rands)


# ------------------------------------------------------------------ full size vs the C oracle
@pytest.fixture(scope="module")
def REF():
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    subprocess.check_call(["make", "-C", os.path.join(root, "oracle"), "-s"])
    C = ctypes.CDLL(os.path.join(root, "oracle", "_build", "libbls_ref.so"))
    C.ref_multi_verify.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p,
                                   ctypes.POINTER(ctypes.c_uint64), ctypes.c_size_t, ctypes.c_int]
    C.ref_hash_to_g2.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t,
                                 ctypes.c_char_p]
    C.ref_sign.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p]
    return C


def test_c2_hash_to_g2_bit_exact_vs_c_oracle(L, G, REF):
    """All 4096 C2 messages: GPU hash_to_G2 (affine, Montgomery bytes) == C oracle."""
    n = 4096
    msgs = [hashlib.sha256(b"h2c-full%d" % i).digest() for i in range(n)]
    dst = b"BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_"
    out = ctypes.create_string_buffer(192 * n)
    G.check(L.gbls_hash_to_g2(G.buf(b"".join(msgs)), G.u32_array(range(0, 32 * n + 1, 32)), n, dst, len(dst), out),
            "h2c")
    step = 7  # the C oracle is ~1 ms per hash: check every 7th message plus the ends
    idx = sorted(set(list(range(0, n, step)) + [n - 1]))
    for i in idx:
        ref = ctypes.create_string_buffer(192)
        REF.ref_hash_to_g2(msgs[i], 32, dst, len(dst), ref)
        assert out.raw[192 * i:192 * (i + 1)] == ref.raw, i


def test_c2_batch_verdicts_vs_c_oracle(B, REF):
    """The GPU verdict of the full 4096-set batch equals the C oracle's verdict on the same
    bytes, for the valid batch, a swapped signature and a flipped scalar-independent message."""
    n = 4096
    sks, msgs, sigs, pks = _workload(B, n, seed=b"vsref")
    rands = [(i * 0x9E3779B97F4A7C15 + 99) % (1 << 64) or 1 for i in range(n)]
    r_arr = (ctypes.c_uint64 * n)(*rands)
    variants = []
    variants.append((msgs, sigs, True))
    bad = list(sigs)
    bad[17] = sigs[18]
    variants.append((msgs, bad, False))
    badm = list(msgs)
    badm[4000] = hashlib.sha256(b"x").digest()
    variants.append((badm, sigs, False))
    for ms, ss, expect in variants:
        gpu = B.Signature.multi_verify(ms, ss, pks, rands)
        ref = REF.ref_multi_verify(b"".join(ms), b"".join(s.raw for s in ss), b"".join(p.raw for p in pks),
                                   r_arr, n, 16)
        assert gpu == bool(ref) == expect
