"""Parity of the kernels behind the headline number (VERDICT r02 "next 2").

Above 32 768 sets per submission the engine switches to its lane-regime kernels
(k_h2c_clear_lane, k_lines_lane, k_mv_g1mul_lane, the c = 13 bucket MSM for segments of
2^16 or more).  These tests run exactly those shapes and compare with the C oracle
(oracle/bls_ref.c) on the same bytes:

* hash_to_G2 of 65 536 messages (lane regime), bit-exact on a seeded sample of 512;
* the bench shape: 16 x 4096-set segments per submission, two submissions in flight on
  two streams, each with its own corrupted segments, every segment's verdict equal to the
  C oracle's on that segment (reference: bls/src/signature.rs:95-129);
* the c = 13 MSM: two 65 536-set segments in one call, signature-side corruption, an
  infinite signature and a zero scalar;
* fast_aggregate_verify golden cases through the batch entry in one call
  (bls/src/signature.rs:77-93).
"""

import ctypes
import hashlib
import json
import os
import random
import subprocess

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DST = b"BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_"


@pytest.fixture(scope="module")
def G():
    from grandine_amd import _lib as G
    G.lib()
    return G


@pytest.fixture(scope="module")
def L(G):
    return G.lib()


@pytest.fixture(scope="module")
def F(G):
    from grandine_amd import factory
    return factory


@pytest.fixture(scope="module")
def REF():
    subprocess.check_call(["make", "-C", os.path.join(ROOT, "oracle"), "-s"])
    C = ctypes.CDLL(os.path.join(ROOT, "oracle", "_build", "libbls_ref.so"))
    C.ref_multi_verify.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p,
                                   ctypes.POINTER(ctypes.c_uint64), ctypes.c_size_t, ctypes.c_int]
    C.ref_hash_to_g2.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t,
                                 ctypes.c_char_p]
    return C


def u64(vals):
    return (ctypes.c_uint64 * len(vals))(*vals)


def _ref_segment(REF, msgs, sigs, pks, rands, b, e):
    return REF.ref_multi_verify(msgs[32 * b:32 * e], sigs[192 * b:192 * e], pks[96 * b:96 * e],
                                u64(rands[b:e]), e - b, 16)


def test_hash_to_g2_lane_regime_65536(G, L, REF):
    n = 1 << 16
    msgs = b"".join(hashlib.sha256(b"h2c-lane/%d" % i).digest() for i in range(n))
    out = ctypes.create_string_buffer(192 * n)
    G.check(L.gbls_hash_to_g2(G.buf(msgs), G.u32_array(range(0, 32 * n + 1, 32)), n, DST, len(DST), out), "h2c")
    rng = random.Random(65536)
    sample = sorted(set(rng.sample(range(n), 512)) | {0, 1, n - 2, n - 1})
    for i in sample:
        ref = ctypes.create_string_buffer(192)
        REF.ref_hash_to_g2(msgs[32 * i:32 * i + 32], 32, DST, len(DST), ref)
        assert out.raw[192 * i:192 * (i + 1)] == ref.raw, i


def _corrupt(msgs, sigs, pks, rands, plan):
    """Apply (kind, set index) corruptions; returns new byte strings / list."""
    m, s, p, r = bytearray(msgs), bytearray(sigs), bytearray(pks), list(rands)
    for kind, i in plan:
        if kind == "swap_sig":  # sets i and i+1 exchange signatures
            s[192 * i:192 * (i + 2)] = sigs[192 * (i + 1):192 * (i + 2)] + sigs[192 * i:192 * (i + 1)]
        elif kind == "flip_msg":
            m[32 * i + 7] ^= 0x10
        elif kind == "wrong_key":
            p[96 * i:96 * (i + 1)] = pks[96 * (i + 1):96 * (i + 2)]
        elif kind == "inf_sig":
            s[192 * i:192 * (i + 1)] = bytes(192)
        elif kind == "inf_key":
            p[96 * i:96 * (i + 1)] = bytes(96)
        else:
            raise ValueError(kind)
    return bytes(m), bytes(s), bytes(p), r


def test_bench_shape_16x4096_two_in_flight(G, L, F, REF):
    """bench.py's default step: 16 independent 4096-set batches as the segments of one
    device submission, two submissions in flight on two streams.  Submission A corrupts
    segments 3 (swapped signatures) and 11 (flipped message); submission B corrupts
    segments 0 (wrong key), 9 (infinite key) and 15 (infinite signature).  Every segment
    verdict equals the C oracle's on that segment's bytes (the oracle runs on the
    corrupted segments and two clean ones of each submission)."""
    import torch
    dev = torch.device("cuda", 0)
    per, nb = 4096, 16
    n = per * nb
    msgs, sigs, pks, rands = F.c2_batch(n, seed=1616)
    plans = {
        "A": [("swap_sig", 3 * per + 100), ("flip_msg", 11 * per + 4000)],
        "B": [("wrong_key", 0 * per + 5), ("inf_key", 9 * per + 77), ("inf_sig", 15 * per + 4095)],
    }
    bad_segs = {"A": {3, 11}, "B": {0, 9, 15}}
    seg = G.u32_array(range(0, n + 1, per))
    inputs, outs, streams = {}, {}, {}
    for k, plan in plans.items():
        m, s, p, r = _corrupt(msgs, sigs, pks, rands, plan)
        inputs[k] = (m, s, p, r)
        streams[k] = torch.cuda.Stream()
    dev_in = {}
    for k, (m, s, p, r) in inputs.items():
        dev_in[k] = [torch.frombuffer(bytearray(x), dtype=torch.uint8).to(dev) for x in (m, s, p)]
        dev_in[k].append(torch.tensor([x - (1 << 64) if x >= 1 << 63 else x for x in r], dtype=torch.int64,
                                      device=dev))
        outs[k] = torch.full((nb,), -1, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    for k in plans:  # both submissions enqueued before either is waited for
        dm, ds, dp, dr = dev_in[k]
        rc = L.gbls_multi_verify_segments_device(dm.data_ptr(), ds.data_ptr(), dp.data_ptr(), dr.data_ptr(), n, seg,
                                                 nb, outs[k].data_ptr(), ctypes.c_void_p(streams[k].cuda_stream))
        assert rc == 0, L.gbls_last_error()
    torch.cuda.synchronize()
    for k in plans:
        got = outs[k].cpu().tolist()
        want = [G.VERIFY_FAIL if j in bad_segs[k] else G.SUCCESS for j in range(nb)]
        assert got == want, (k, got)
        m, s, p, r = inputs[k]
        for j in sorted(bad_segs[k] | {1, 14}):
            ref = _ref_segment(REF, m, s, p, r, j * per, (j + 1) * per)
            assert (got[j] == G.SUCCESS) == bool(ref), (k, j, got[j], ref)


def test_msm_c13_two_large_segments(G, L, F, REF):
    """the c = 13 bucket MSM (per-window trees, segments of >= 2^16 sets) with
    two segments in one launch: a signature-side corruption in segment 1, then an
    infinite signature in segment 0, then a zero scalar (fails closed).  The corrupted
    segment's verdict is checked against the C oracle too."""
    per = 1 << 16
    n = 2 * per
    msgs, sigs, pks, rands = F.c2_batch(n, seed=1313)
    seg = G.u32_array([0, per, n])
    v = G.i32_array(2)
    G.check(L.gbls_multi_verify_segments(msgs, sigs, pks, u64(rands), n, seg, 2, v), "segs")
    assert (v[0], v[1]) == (G.SUCCESS, G.SUCCESS)
    m, s, p, r = _corrupt(msgs, sigs, pks, rands, [("swap_sig", per + 30000)])
    G.check(L.gbls_multi_verify_segments(m, s, p, u64(r), n, seg, 2, v), "segs")
    assert (v[0], v[1]) == (G.SUCCESS, G.VERIFY_FAIL)
    assert _ref_segment(REF, m, s, p, r, per, n) == 0
    m, s, p, r = _corrupt(msgs, sigs, pks, rands, [("inf_sig", 12345)])
    G.check(L.gbls_multi_verify_segments(m, s, p, u64(r), n, seg, 2, v), "segs")
    assert (v[0], v[1]) == (G.VERIFY_FAIL, G.SUCCESS)
    r0 = list(rands)
    r0[per + 1] = 0
    G.check(L.gbls_multi_verify_segments(msgs, sigs, pks, u64(r0), n, seg, 2, v), "segs")
    assert (v[0], v[1]) == (G.SUCCESS, G.VERIFY_FAIL)


def test_fast_aggregate_verify_golden_batch(G, L):
    """Every golden fast_aggregate_verify case (infinite signature, signature not in G2,
    infinity member keys, no keys, keys cancelling) as the messages of ONE batch call."""
    from grandine_amd import bls as B
    with open(os.path.join(ROOT, "tests", "golden", "fast_aggregate_verify.json")) as fh:
        cases = json.load(fh)["cases"]
    sigs, msgs, moff, keys, koff = [], b"", [0], [], [0]
    for c in cases:
        sigs.append(B.Signature.try_from(bytes.fromhex(c["sig"])).raw)
        msgs += bytes.fromhex(c["msg"])
        moff.append(len(msgs))
        for h in c["pks"]:
            if h == "c0" + "00" * 47:
                keys.append(bytes(96))
            else:
                st, raw = B.decompress_public_keys([bytes.fromhex(h)], validate=False)[0]
                assert st == 0
                keys.append(raw)
        koff.append(len(keys))
    m = len(cases)
    v = G.i32_array(m)
    G.check(L.gbls_fast_aggregate_verify_batch(G.buf(b"".join(sigs)), G.buf(msgs), G.u32_array(moff),
                                               G.buf(b"".join(keys)), G.u32_array(koff), m, v), "fav_batch")
    for i, c in enumerate(cases):
        assert (v[i] == G.SUCCESS) == c["expect"], c["note"]


def test_fast_aggregate_verify_grouped_matches_single_checks(G, L, F):
    """Batches of >= 2048 independent checks take the grouped form (gbls_capi.hip
    grouped_verdicts: random G1-side weights, eight checks per final exponentiation, every
    member of a failing or flagged group re-checked on its own).  On one 4096-check batch with
    dense and clustered failures -- 20 % flipped messages, one group of eight all invalid, and
    every golden fast_aggregate_verify case (infinite signature, signature not in G2, missing /
    no / cancelling / infinity member keys) placed at group boundaries and inside groups --
    each verdict equals the per-check form's (the same bytes in calls of < 2048 checks) and
    the construction's expectation."""
    from grandine_amd import bls as B
    n = 4096
    msgs, sigs, pks, _ = F.c2_batch(n, seed=3030)
    rng = random.Random(3030)
    sig_l = [sigs[192 * i:192 * (i + 1)] for i in range(n)]
    msg_l = [msgs[32 * i:32 * (i + 1)] for i in range(n)]
    key_l = [[pks[96 * i:96 * (i + 1)]] for i in range(n)]
    expect = [True] * n
    for i in list(range(40, 48)) + rng.sample(range(64, n), n // 5):  # flipped messages
        m = bytearray(msg_l[i])
        m[3] ^= 0x40
        msg_l[i] = bytes(m)
        expect[i] = False
    with open(os.path.join(ROOT, "tests", "golden", "fast_aggregate_verify.json")) as fh:
        cases = json.load(fh)["cases"]
    slots = [8 * g + (g % 8) for g in range(100, 100 + 6 * len(cases))]  # every position in a group
    for j, i in enumerate(slots):
        c = cases[j % len(cases)]
        sig_l[i] = B.Signature.try_from(bytes.fromhex(c["sig"])).raw
        msg_l[i] = bytes.fromhex(c["msg"])
        keys = []
        for h in c["pks"]:
            if h == "c0" + "00" * 47:
                keys.append(bytes(96))
            else:
                st, raw = B.decompress_public_keys([bytes.fromhex(h)], validate=False)[0]
                assert st == 0
                keys.append(raw)
        key_l[i] = keys
        expect[i] = c["expect"]
    # two checks in ONE group whose UNWEIGHTED pairing products cancel -- same key
    # and message, signatures sigma + D and sigma - D (D in G2).  Each is invalid, but their
    # product e(pk, H)^2 e(-g1, 2 sigma) is 1, so only the secret r_i weights (on both G1 sides
    # of each check) can make the group fail
    P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB

    def neg(pt):  # affine G2 point, Montgomery bytes: y -> p - y per Fp component
        y0, y1 = (int.from_bytes(pt[96 + 48 * k:144 + 48 * k], "little") for k in range(2))
        return pt[:96] + b"".join(((P - y) % P).to_bytes(48, "little") for y in (y0, y1))

    def add(a, b):
        out = ctypes.create_string_buffer(192)
        G.check(L.gbls_g2_aggregate(G.buf(a + b), 2, out), "g2 sum")
        return out.raw

    D, sigma = sig_l[5], sig_l[16]
    sig_l[16], sig_l[17] = add(sigma, D), add(sigma, neg(D))
    msg_l[17], key_l[17] = msg_l[16], key_l[16]
    expect[16] = expect[17] = False

    def run(b, e):
        moff, koff, keys = [0], [0], []
        for i in range(b, e):
            moff.append(moff[-1] + len(msg_l[i]))
            keys += key_l[i]
            koff.append(len(keys))
        v = G.i32_array(e - b)
        G.check(L.gbls_fast_aggregate_verify_batch(G.buf(b"".join(sig_l[b:e])), G.buf(b"".join(msg_l[b:e])),
                                                   G.u32_array(moff), G.buf(b"".join(keys) or bytes(96)),
                                                   G.u32_array(koff), e - b, v), "fav_batch")
        return [v[k] for k in range(e - b)]

    grouped = run(0, n)
    single = []
    for b in range(0, n, 1024):
        single += run(b, b + 1024)
    assert grouped == single
    assert [x == G.SUCCESS for x in grouped] == expect
    assert grouped[16] == grouped[17] == G.VERIFY_FAIL  # the cancelling pair
    # GBLS_INIT_PER_CHECK: the same 4096-check batch in ONE call with
    # grouping off (a Miller product and final exponentiation per check) -> the same verdicts
    PER_CHECK = 0x400
    assert L.gbls_init(0, PER_CHECK) == G.SUCCESS
    try:
        per_check = run(0, n)
    finally:
        assert L.gbls_init(0, 0) == G.SUCCESS
    assert per_check == grouped


def test_grouped_device_call_is_asynchronous(G, L, F):
    """the grouped form's second round (member verdicts, re-checks of
    failed groups) runs on the device, so gbls_fast_aggregate_verify_indexed_device returns
    before its stream has finished, and its verdicts (checked after the stream sync) are right:
    4096 sync-committee-shaped checks over registry indices, 1 % invalid."""
    import numpy as np
    import time
    import torch
    dev = torch.device("cuda", 0)
    k, m = 64, 4096
    sks, comp = F.registry(1 << 12, seed=b"async-fav")
    first = G.lib().gbls_registry_size()
    assert not F.load_registry(comp, first).any()
    rng = np.random.default_rng(11)
    committee = rng.choice(1 << 12, size=k, replace=False).astype(np.uint32)
    ssum = sum(sks[int(i)] for i in committee) % F.R_ORDER
    msgs = F.messages(m, b"async-fav")
    sigs = bytearray(F.sign([ssum] * m, msgs))
    bad = sorted(rng.choice(m, size=m // 100, replace=False).tolist())
    wrong = F.sign([(ssum + 1) % F.R_ORDER], msgs[:32])
    for i in bad:
        sigs[192 * i:192 * i + 192] = wrong
    d_msgs = torch.frombuffer(bytearray(msgs), dtype=torch.uint8).to(dev)
    d_sigs = torch.frombuffer(sigs, dtype=torch.uint8).to(dev)
    d_idx = torch.from_numpy((np.tile(committee, m) + first).astype(np.uint32).view(np.int32)).to(dev)
    d_off = torch.from_numpy(np.arange(0, k * m + 1, k, dtype=np.uint32).view(np.int32)).to(dev)
    d_v = torch.full((m,), -1, dtype=torch.int32, device=dev)
    s = torch.cuda.Stream()
    ptr = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    with torch.cuda.stream(s):
        # warm (buffers grown), then the measured call
        G.check(L.gbls_fast_aggregate_verify_indexed_device(ptr(d_sigs), ptr(d_msgs), ptr(d_idx), ptr(d_off), m,
                                                            ptr(d_v), ctypes.c_void_p(s.cuda_stream)), "warm")
        s.synchronize()
        d_v.fill_(-1)
        t0 = time.perf_counter()
        G.check(L.gbls_fast_aggregate_verify_indexed_device(ptr(d_sigs), ptr(d_msgs), ptr(d_idx), ptr(d_off), m,
                                                            ptr(d_v), ctypes.c_void_p(s.cuda_stream)), "fav")
        t_call = time.perf_counter() - t0
        pending = not s.query()
        s.synchronize()
        t_all = time.perf_counter() - t0
    assert pending, "the device call returned after its stream had finished (host-synchronous)"
    want = np.zeros(m, dtype=np.int32)
    want[bad] = G.VERIFY_FAIL
    assert (d_v.cpu().numpy() == want).all()
    assert t_call < t_all, (t_call, t_all)
