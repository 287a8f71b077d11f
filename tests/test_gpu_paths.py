"""On-device coverage of the paths and BASELINE configs beyond C2 (VERDICT r01 "next 1"):

* the multi-GPU kernels on one GPU: per-shard Miller partials + one final
  exponentiation over k partials (bench.py's RCCL flow without the all-gather);
* C3 -- sync-committee fast_aggregate_verify, 512 keys x 10,000 messages, 1 % invalid;
* C4 -- an epoch of 2,048 committees over a 2^20-key registry: indexed aggregation
  (Triple::verify_aggregate) + multi_verify of the 2,048 aggregate sets;
* C5 -- one GPU's shard of the Holesky-scale stress: 2^17 sets with key indices drawn
  from a 1.7M-key registry;
* robustness: zero scalars fail closed, bad offsets are argument errors, concurrent
  callers on many threads and streams, per-set verdicts by GPU bisection, and the
  multi-engine sharding of host calls (several engines on one GPU, in a subprocess).

Every verdict is checked against the construction (which sets were corrupted) and, on
seeded samples, against the C oracle (oracle/bls_ref.c) on the same bytes; aggregated
keys are checked bit-exact against (sum of secret keys) * G1.
"""

import ctypes
import hashlib
import json
import os
import subprocess
import sys
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


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
    C.ref_multi_verify_partial.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p,
                                           ctypes.POINTER(ctypes.c_uint64), ctypes.c_size_t, ctypes.c_char_p]
    C.ref_verify.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p]
    C.ref_sk_to_pk.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
    return C


def u64(vals):
    return (ctypes.c_uint64 * len(vals))(*vals)


# ------------------------------------------------------------------ multi-GPU kernels on one GPU
@pytest.fixture(scope="module")
def torch_dev():
    import torch
    return torch, torch.device("cuda", 0)


def _dev(torch, dev, b):
    return torch.frombuffer(bytearray(b), dtype=torch.uint8).to(dev)


def _sharded_verdict(torch, dev, L, G, msgs, sigs, pks, rands, k, tamper=None):
    """Split the sets into k contiguous shards (k may exceed n: empty shards), one partial
    each through gbls_multi_verify_partials_device, then one final exponentiation over
    the k partials (gbls_final_verify_partials_device, nparts = k)."""
    n = len(rands)
    parts = torch.zeros(k * 576, dtype=torch.uint8, device=dev)
    errs = torch.zeros(k, dtype=torch.int32, device=dev)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    for j in range(k):
        b, e = n * j // k, n * (j + 1) // k
        m = _dev(torch, dev, msgs[32 * b:32 * e] or b"\0")
        s = _dev(torch, dev, sigs[192 * b:192 * e] or b"\0")
        p = _dev(torch, dev, pks[96 * b:96 * e] or b"\0")
        r = torch.tensor([x - (1 << 64) if x >= 1 << 63 else x for x in rands[b:e]] or [1],
                         dtype=torch.int64, device=dev)
        seg = G.u32_array([0, e - b])
        rc = L.gbls_multi_verify_partials_device(m.data_ptr(), s.data_ptr(), p.data_ptr(), r.data_ptr(),
                                                 e - b, seg, 1, parts.data_ptr() + 576 * j,
                                                 errs.data_ptr() + 4 * j, st)
        assert rc == 0, L.gbls_last_error()
        torch.cuda.synchronize()
    if tamper is not None:
        parts[576 * tamper] ^= 1
    v = torch.full((1,), -1, dtype=torch.int32, device=dev)
    assert L.gbls_final_verify_partials_device(parts.data_ptr(), errs.data_ptr(), k, 1, v.data_ptr(), st) == 0
    torch.cuda.synchronize()
    return int(v.item())


def test_partials_k_shards_c2(G, L, F, REF, torch_dev):
    torch, dev = torch_dev
    n = 4096
    msgs, sigs, pks, rands = F.c2_batch(n, seed=11)
    ref = REF.ref_multi_verify(msgs, sigs, pks, u64(rands), n, 16)
    assert ref == 1
    for k in (1, 2, 3, 8):
        assert _sharded_verdict(torch, dev, L, G, msgs, sigs, pks, rands, k) == G.SUCCESS, k
    assert _sharded_verdict(torch, dev, L, G, msgs, sigs, pks, rands, 3, tamper=2) == G.VERIFY_FAIL
    bad = bytearray(sigs)
    bad[192 * 3000:192 * 3001] = sigs[192 * 3001:192 * 3002]
    bad = bytes(bad)
    assert REF.ref_multi_verify(msgs, bad, pks, u64(rands), n, 16) == 0
    for k in (2, 8):
        assert _sharded_verdict(torch, dev, L, G, msgs, bad, pks, rands, k) == G.VERIFY_FAIL, k


def test_partials_more_shards_than_sets(G, L, torch_dev):
    """k > n: the empty shards contribute identity partials (empty shard)."""
    torch, dev = torch_dev
    from grandine_amd import factory as F
    msgs, sigs, pks, rands = F.c2_batch(3, seed=12)
    assert _sharded_verdict(torch, dev, L, G, msgs, sigs, pks, rands, 8) == G.SUCCESS
    bad = msgs[:32] + bytes(32) + msgs[64:]
    assert _sharded_verdict(torch, dev, L, G, bad, sigs, pks, rands, 8) == G.VERIFY_FAIL


def test_partial_bytes_match_c_oracle_partial_verdict(G, L, F, REF, torch_dev):
    """A GPU shard partial combined with a C-oracle shard partial verifies: both are
    Miller products of the same pairing equation (any correct Fp12 chain; SURVEY 8(a)
    contract 9), so the cross product must pass the final exponentiation."""
    torch, dev = torch_dev
    n = 64
    msgs, sigs, pks, rands = F.c2_batch(n, seed=13)
    h = n // 2
    cpart = ctypes.create_string_buffer(576)
    assert REF.ref_multi_verify_partial(msgs[32 * h:], sigs[192 * h:], pks[96 * h:], u64(rands[h:]), n - h, cpart) == 0
    parts = torch.zeros(2 * 576, dtype=torch.uint8, device=dev)
    errs = torch.zeros(2, dtype=torch.int32, device=dev)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    m, s, p = _dev(torch, dev, msgs[:32 * h]), _dev(torch, dev, sigs[:192 * h]), _dev(torch, dev, pks[:96 * h])
    r = torch.tensor([x - (1 << 64) if x >= 1 << 63 else x for x in rands[:h]], dtype=torch.int64, device=dev)
    assert L.gbls_multi_verify_partials_device(m.data_ptr(), s.data_ptr(), p.data_ptr(), r.data_ptr(), h,
                                               G.u32_array([0, h]), 1, parts.data_ptr(), errs.data_ptr(), st) == 0
    parts[576:] = torch.frombuffer(bytearray(cpart.raw), dtype=torch.uint8).to(dev)
    v = torch.full((1,), -1, dtype=torch.int32, device=dev)
    assert L.gbls_final_verify_partials_device(parts.data_ptr(), errs.data_ptr(), 2, 1, v.data_ptr(), st) == 0
    torch.cuda.synchronize()
    assert int(v.item()) == G.SUCCESS


# ------------------------------------------------------------------ robustness of the ABI
def test_zero_scalar_fails_closed(G, L, F):
    """a zero scalar would drop its set from the combination; every path fails
    the batch instead (device segments path included)."""
    msgs, sigs, pks, rands = F.c2_batch(6, seed=14)
    bad_sigs = sigs[:192 * 2] + sigs[192 * 3:192 * 4] + sigs[192 * 3:]  # set 2 invalid
    r0 = list(rands)
    r0[2] = 0
    v = G.i32_array(2)
    off = G.u32_array([0, 3, 6])
    G.check(L.gbls_multi_verify_segments(msgs, bad_sigs, pks, u64(r0), 6, off, 2, v), "segs")
    assert (v[0], v[1]) == (G.VERIFY_FAIL, G.SUCCESS)
    G.check(L.gbls_multi_verify_segments(msgs, sigs, pks, u64(r0), 6, off, 2, v), "segs")
    assert (v[0], v[1]) == (G.VERIFY_FAIL, G.SUCCESS)
    assert L.gbls_multi_verify(msgs, sigs, pks, u64(r0), 6) == G.VERIFY_FAIL
    assert L.gbls_multi_verify(msgs, sigs, pks, u64(rands), 6) == G.SUCCESS


def test_bad_segment_offsets_are_argument_errors(G, L, F):
    msgs, sigs, pks, rands = F.c2_batch(4, seed=15)
    v = G.i32_array(2)
    for off in ([1, 2, 4], [0, 3, 2], [0, 2, 5]):
        v[0] = v[1] = 0
        rc = L.gbls_multi_verify_segments(msgs, sigs, pks, u64(rands), 4, G.u32_array(off), 2, v)
        assert rc == G.VERIFY_FAIL and L.gbls_last_error() == 102, off
        assert (v[0], v[1]) == (G.VERIFY_FAIL, G.VERIFY_FAIL)


def test_hash_to_g2_default_dst_and_argument_errors(G, L):
    """gbls_hash_to_g2 with dst == NULL uses the POP scheme's DST (the same points as passing it
    explicitly); NULL with a nonzero length, or a NULL message array, is an argument error
    (it crashed in upload before r04)."""
    dst = b"BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_"
    n = 3
    msgs = bytes(range(32 * n))
    off = G.u32_array(range(0, 32 * n + 1, 32))
    a = (ctypes.c_uint8 * (192 * n))()
    b = (ctypes.c_uint8 * (192 * n))()
    G.check(L.gbls_hash_to_g2(G.buf(msgs), off, n, dst, len(dst), a), "explicit dst")
    G.check(L.gbls_hash_to_g2(G.buf(msgs), off, n, None, 0, b), "default dst")
    assert bytes(a) == bytes(b)
    assert L.gbls_hash_to_g2(G.buf(msgs), off, n, None, 5, b) == G.VERIFY_FAIL and L.gbls_last_error() == 102
    assert L.gbls_hash_to_g2(None, off, n, dst, len(dst), b) == G.VERIFY_FAIL and L.gbls_last_error() == 102


def test_concurrent_callers_threads_and_streams(G, L, F, torch_dev):
    """many threads call in at once.  8 host threads x 6 calls (host-pointer
    and device-pointer on per-thread streams), a mix of valid and corrupted batches; every
    verdict must match its own batch."""
    torch, dev = torch_dev
    batches = []
    for t in range(8):
        msgs, sigs, pks, rands = F.c2_batch(96 + 16 * t, seed=100 + t)
        bad = bytearray(msgs)
        bad[5] ^= 0x40
        batches.append((msgs, bytes(bad), sigs, pks, rands))
    errors = []

    def worker(t):
        try:
            torch.cuda.set_device(0)
            msgs, bad, sigs, pks, rands = batches[t]
            n = len(rands)
            stream = torch.cuda.Stream()
            dm, db, ds, dp = (_dev(torch, dev, x) for x in (msgs, bad, sigs, pks))
            dr = torch.tensor([x - (1 << 64) if x >= 1 << 63 else x for x in rands], dtype=torch.int64, device=dev)
            seg = G.u32_array([0, n])
            for it in range(6):
                expect_ok = (it + t) % 2 == 0
                if it % 3 == 2:
                    v = torch.full((1,), -1, dtype=torch.int32, device=dev)
                    # the fill ran on this thread's current stream: order it before the call's
                    # stream (an unordered fill can land after the verdict and read as -1)
                    stream.wait_stream(torch.cuda.current_stream())
                    with torch.cuda.stream(stream):
                        rc = L.gbls_multi_verify_segments_device((dm if expect_ok else db).data_ptr(), ds.data_ptr(),
                                                                 dp.data_ptr(), dr.data_ptr(), n, seg, 1, v.data_ptr(),
                                                                 ctypes.c_void_p(stream.cuda_stream))
                    stream.synchronize()
                    got = int(v.item()) if rc == 0 else -rc
                else:
                    got = L.gbls_multi_verify(msgs if expect_ok else bad, sigs, pks, u64(rands), n)
                if got != (G.SUCCESS if expect_ok else G.VERIFY_FAIL):
                    errors.append((t, it, got))
        except Exception as e:  # noqa: BLE001
            errors.append((t, repr(e)))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errors, errors


def test_bisection_finds_planted_bad_sets(G, L, F):
    """f2: per-set verdicts of a 4096-set batch with 5 planted bad sets (wrong message,
    swapped signature, infinite key, zero scalar, wrong key)."""
    n = 4096
    msgs, sigs, pks, rands = F.c2_batch(n, seed=16)
    m, s, p, r = bytearray(msgs), bytearray(sigs), bytearray(pks), list(rands)
    m[32 * 17] ^= 1
    s[192 * 1000:192 * 1001] = sigs[192 * 1001:192 * 1002]
    p[96 * 2048:96 * 2049] = bytes(96)
    r[3333] = 0
    p[96 * 4095:96 * 4096] = pks[0:96]
    bad = {17, 1000, 2048, 3333, 4095}
    v = G.i32_array(n)
    G.check(L.gbls_multi_verify_bisect(bytes(m), bytes(s), bytes(p), None, None, u64(r), n, v), "bisect")
    got = {i for i in range(n) if v[i] != G.SUCCESS}
    assert got == bad
    G.check(L.gbls_multi_verify_bisect(msgs, sigs, pks, None, None, u64(rands), n, v), "bisect")
    assert all(v[i] == G.SUCCESS for i in range(n))


def test_multi_engine_sharding_subprocess():
    """Several engines on the one GPU (gbls_init flags = 3): host calls shard one large
    batch into per-engine Miller partials + one final exponentiation, and spread segments
    over the engines (the single-process multi-device path)."""
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "gpu_replicas.py")], capture_output=True,
                         text=True, timeout=600)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-2000:]
    res = json.loads(out.stdout.strip().splitlines()[-1])
    assert res["engines"] == 3
    assert res == {"engines": 3, "big_valid": 0, "big_bad": 5, "segs": [0, 5, 0, 0, 5, 0], "bisect": [7, 3000],
                   "registry": 0}


def test_bucket_msm_parity_subprocess():
    """n1: the bucket-MSM path for S (k_msm.hip), forced on every batch size
    (GBLS_MSM_MIN=1): golden multi_verify verdicts, and 4096-set batches (valid, swapped
    signature, infinite signature, crowded and near-empty buckets) equal to the C
    oracle's verdicts; a zero scalar fails closed."""
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "gpu_msm.py")], capture_output=True,
                         text=True, timeout=600)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-2000:]
    res = json.loads(out.stdout.strip().splitlines()[-1])
    assert all(res["golden"]), res
    for name, gpu, ref in res["c2"]:
        assert gpu == ref, (name, gpu, ref)
    assert [x[1] for x in res["c2"]] == [True, False, False, True, True]
    assert res["segments"] == [0, 5, 0, 5, 0]
    assert res["zero_scalar"] == 5


@pytest.mark.parametrize("knobs", [["GBLS_ML_DMA=1"], ["GBLS_ML_R28=0"], ["GBLS_LANE_R28=0"], ["GBLS_ML_KARA=1"],
                                   ["GBLS_LANE_MIN=1"], ["GBLS_LANE_MIN=1", "GBLS_CLEAR_STAGED=1"]],
                         ids=["ml-lds-dma", "ml-radix32", "lanes-radix32", "ml-karatsuba", "lanes-everywhere",
                              "clear-staged"])
def test_kernel_variants_subprocess(knobs):
    """The non-default kernel forms an operator can select (k_ml_group28 with the line staged
    in LDS by DMA loads; the 32-bit-limb k_ml_group; the 32-bit-limb line / cofactor lanes; the
    lane forms at every launch size above the W4 regime, partial waves included; the same with
    the staged cofactor clearing, GBLS_CLEAR_STAGED=1):
    golden multi_verify verdicts, 4096-set batches equal to the C oracle's, and a 4-segment
    batch that flags exactly its corrupted segment (tests/gpu_knobs.py, its own engine)."""
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "gpu_knobs.py")] + knobs,
                         capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-2000:]
    res = json.loads(out.stdout.strip().splitlines()[-1])
    assert res["knobs"] == knobs and all(res["golden"]), res
    for name, gpu, ref in res["c2"]:
        assert gpu == ref, (name, gpu, ref)
    assert [x[1] for x in res["c2"]] == [True, False, False]
    assert res["segments"] == [0, 0, 5, 0]


def test_sliced_lines_subprocess():
    """Event-sliced Miller lines (GBLS_LINE_BUDGET_MB=16: a 4096-set batch in slices of
    a few events, the running points in HBM between slices): single-batch verdicts equal
    the C oracle's, and a 4-segment batch flags exactly the segment with swapped
    signatures."""
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "gpu_sliced.py")], capture_output=True,
                         text=True, timeout=600)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-2000:]
    res = json.loads(out.stdout.strip().splitlines()[-1])
    assert res["ref"] == [1, 0], res
    assert res["single"] == [0, 5], res
    assert [s[1:] for s in res["segments"]] == [[0, 0, 0, 0], [0, 0, 5, 0]], res


# ------------------------------------------------------------------ registry (C4 / C5 shapes)
N_REG = 1_700_000


@pytest.fixture(scope="module")
def registry(G, L, F):
    sks, comp = F.registry(N_REG, seed=b"holesky")
    st = F.load_registry(comp)
    assert not st.any(), "every registry key must decompress and validate"
    assert L.gbls_registry_size() >= N_REG
    return sks, comp


def test_registry_invalid_keys_and_growth(G, L, F, registry):
    sks, comp = registry
    junk = [bytes(48), b"\xc0" + bytes(47), comp[:48][:47] + bytes([comp[47] ^ 1])]
    base = N_REG + 10
    st = F.load_registry(b"".join(junk), first=base)
    assert list(st) == [G.BAD_ENCODING, G.PK_IS_INFINITY, st[2]] and st[2] != 0
    assert L.gbls_registry_size() == base + 3
    # gaps and invalid entries are infinity: a set using them fails
    msgs = F.messages(1, b"gap")
    sig = F.sign([sks[0]], msgs)
    for idx in (N_REG + 1, base, base + 1, 1 << 31):
        assert L.gbls_multi_verify_indexed(msgs, sig, G.u32_array([idx]), None, u64([5]), 1) == G.VERIFY_FAIL
    assert L.gbls_multi_verify_indexed(msgs, sig, G.u32_array([0]), None, u64([5]), 1) == G.SUCCESS


def test_registry_aggregates_with_gap_or_invalid_member_fail(G, L, F, registry):
    """an aggregate over registry indices that names a gap slot or an
    invalid key must fail, not verify as if the member were absent (the reference fails
    the check when a member key does not decompress, helper_functions/src/predicates.rs:130).
    Covers the aggregation entry, multi_verify_indexed with pk_off (workgroup and row
    kernels: 1 and 200 segments), fast_aggregate_verify_indexed, and the fused finish."""
    sks, comp = registry
    base = N_REG + 10  # test_registry_invalid_keys_and_growth: base = invalid, base + 1 = infinity
    F.load_registry(bytes(48), first=base)  # (idempotent when run alone: an invalid key at base)
    gap, invalid = N_REG + 1, base
    msgs = F.messages(1, b"gap-agg")
    sig = F.sign([sks[0]], msgs)  # signed by member 0 alone
    for other in (gap, invalid):
        idx = G.u32_array([0, other])
        off = G.u32_array([0, 2])
        agg = ctypes.create_string_buffer(96)
        st = G.i32_array(1)
        G.check(L.gbls_g1_aggregate_indexed(idx, off, 1, agg, st), "aggregate_indexed")
        assert st[0] == G.BAD_ENCODING, other
        assert L.gbls_multi_verify_indexed(msgs, sig, idx, off, u64([7]), 1) == G.VERIFY_FAIL, other
        v = G.i32_array(1)
        G.check(L.gbls_fast_aggregate_verify_indexed(sig, msgs, G.u32_array([0, 32]), idx, off, 1, v), "fav")
        assert v[0] == G.VERIFY_FAIL, other
        comp_sig = ctypes.create_string_buffer(96)
        G.check(L.gbls_g2_compress(sig, 1, comp_sig), "compress")
        sst = G.i32_array(1)
        assert L.gbls_multi_verify_compressed(msgs, comp_sig, None, idx, off, u64([7]), 1, sst) == G.VERIFY_FAIL
    # the same member alone verifies (the failure above is the gap / invalid member)
    assert L.gbls_multi_verify_indexed(msgs, sig, G.u32_array([0]), G.u32_array([0, 1]), u64([7]), 1) == G.SUCCESS
    # row kernel (>= 128 segments): 200 two-member committees, one with a gap member
    m = 200
    ms = F.messages(m, b"gap-rows")
    sums = [(sks[2 * i] + sks[2 * i + 1]) % F.R_ORDER for i in range(m)]
    sigs = F.sign(sums, ms)
    idx = list(range(2 * m))
    idx[2 * 123 + 1] = gap
    st = G.i32_array(m)
    agg = ctypes.create_string_buffer(96 * m)
    G.check(L.gbls_g1_aggregate_indexed(G.u32_array(idx), G.u32_array(range(0, 2 * m + 1, 2)), m, agg, st), "agg")
    assert [i for i in range(m) if st[i] != 0] == [123]
    v = G.i32_array(m)
    G.check(L.gbls_fast_aggregate_verify_indexed(sigs, ms, G.u32_array(range(0, 32 * m + 1, 32)), G.u32_array(idx),
                                                 G.u32_array(range(0, 2 * m + 1, 2)), m, v), "fav rows")
    assert [i for i in range(m) if v[i] != 0] == [123]


def test_c4_epoch_aggregation_and_verify(G, L, F, REF, registry):
    """C4: 32 x 64 committees over a 2^20-key registry (sizes 511/512)."""
    sks, comp = registry
    ncom, nact = 2048, 1_048_000
    idx, off = F.committees(nact, ncom, seed=4)
    msgs = F.messages(ncom, b"c4")
    sigs, sums = F.committee_signatures(sks, idx, off, msgs)
    idx_c = idx.ctypes.data_as(ctypes.c_void_p)
    off_c = off.ctypes.data_as(ctypes.c_void_p)
    # aggregation bit-exact: sum of committee keys == (sum of committee sks) * G1
    agg = ctypes.create_string_buffer(96 * ncom)
    st = G.i32_array(ncom)
    G.check(L.gbls_g1_aggregate_indexed(idx_c, off_c, ncom, agg, st), "aggregate_indexed")
    assert all(st[i] == 0 for i in range(ncom))
    assert agg.raw == F.public_keys(sums)
    for c in (0, 777, 2047):  # and against the C oracle's sk -> pk
        ref = ctypes.create_string_buffer(96)
        REF.ref_sk_to_pk(sums[c].to_bytes(32, "big"), ref)
        assert agg.raw[96 * c:96 * c + 96] == ref.raw
    rands = F.rands(ncom, 4)
    assert L.gbls_multi_verify_indexed(msgs, sigs, idx_c, off_c, u64(rands), ncom) == G.SUCCESS
    ref = REF.ref_multi_verify(msgs, sigs, agg.raw, u64(rands), ncom, 16)
    assert ref == 1
    bad = bytearray(sigs)
    bad[192 * 5:192 * 6] = sigs[192 * 6:192 * 7]
    assert L.gbls_multi_verify_indexed(msgs, bytes(bad), idx_c, off_c, u64(rands), ncom) == G.VERIFY_FAIL
    # a committee missing one member fails, and bisection names exactly that committee
    idx2 = idx.copy()
    idx2[int(off[100])] = idx2[int(off[100]) + 1]
    v = G.i32_array(ncom)
    G.check(L.gbls_multi_verify_bisect(msgs, sigs, None, idx2.ctypes.data_as(ctypes.c_void_p), off_c, u64(rands), ncom,
                                       v), "bisect")
    assert [i for i in range(ncom) if v[i] != 0] == [100]


def test_c5_shard_indexed_131072(G, L, F, REF, registry):
    """C5 per-GPU shard: 2^20 sets over 8 GPUs = 2^17 sets per GPU, key indices drawn
    uniformly from the 1.7M-key registry, distinct messages."""
    sks, comp = registry
    n = 1 << 17
    rng = np.random.default_rng(5)
    idx = rng.integers(0, N_REG, size=n, dtype=np.uint32)
    msgs = F.messages(n, b"c5")
    sigs = F.sign([sks[int(i)] for i in idx], msgs)
    rands = F.rands(n, 5)
    idx_c = idx.ctypes.data_as(ctypes.c_void_p)
    assert L.gbls_multi_verify_indexed(msgs, sigs, idx_c, None, u64(rands), n) == G.SUCCESS
    bad = bytearray(msgs)
    bad[32 * 99999] ^= 0x80
    assert L.gbls_multi_verify_indexed(bytes(bad), sigs, idx_c, None, u64(rands), n) == G.VERIFY_FAIL
    # C oracle on a seeded 2048-set slice of the same bytes
    pk_pts = F.public_keys([sks[int(i)] for i in idx[:2048]])
    assert REF.ref_multi_verify(msgs[:32 * 2048], sigs[:192 * 2048], pk_pts, u64(rands[:2048]), 2048, 16) == 1
    assert L.gbls_multi_verify_indexed(msgs[:32 * 2048], sigs[:192 * 2048], idx_c, None, u64(rands[:2048]),
                                       2048) == G.SUCCESS


def test_c5_full_2pow20_sliced_accept_and_reject(G, L, F, REF, registry):
    """C5 at full size on one GPU: 2^20 sets from the 1.7M registry, whose Miller lines
    exceed the 4 GB line budget and run in event slices.  Accepts the valid batch and
    rejects one flipped message and, separately, one swapped signature pair near the end;
    the C oracle agrees on a 2048-set slice around each corruption."""
    sks, comp = registry
    n = 1 << 20
    rng = np.random.default_rng(20)
    idx = rng.integers(0, N_REG, size=n, dtype=np.uint32)
    msgs = F.messages(n, b"c5-full")
    sigs = F.sign([sks[int(i)] for i in idx], msgs)
    rands = F.rands(n, 20)
    idx_c = idx.ctypes.data_as(ctypes.c_void_p)
    assert L.gbls_multi_verify_indexed(msgs, sigs, idx_c, None, u64(rands), n) == G.SUCCESS
    bad_m = bytearray(msgs)
    bad_m[32 * 700001 + 3] ^= 0x01
    bad_m = bytes(bad_m)
    assert L.gbls_multi_verify_indexed(bad_m, sigs, idx_c, None, u64(rands), n) == G.VERIFY_FAIL
    bad_s = bytearray(sigs)
    j = n - 10
    bad_s[192 * j:192 * (j + 2)] = sigs[192 * (j + 1):192 * (j + 2)] + sigs[192 * j:192 * (j + 1)]
    bad_s = bytes(bad_s)
    assert L.gbls_multi_verify_indexed(msgs, bad_s, idx_c, None, u64(rands), n) == G.VERIFY_FAIL
    # the C oracle and the engine on 2048-set slices of the same bytes: a clean slice (accept,
    # so the full-size accept above is not pinned by device-signed data alone) and the slice
    # around each corruption (reject)
    for (m_, s_, at, want) in ((msgs, sigs, 300000, 1), (bad_m, sigs, 700001 - 1000, 0), (msgs, bad_s, n - 2048, 0)):
        b, e = at, at + 2048
        pk_pts = F.public_keys([sks[int(i)] for i in idx[b:e]])
        assert REF.ref_multi_verify(m_[32 * b:32 * e], s_[192 * b:192 * e], pk_pts, u64(rands[b:e]), e - b, 16) == want
        sl = np.ascontiguousarray(idx[b:e])
        assert L.gbls_multi_verify_indexed(m_[32 * b:32 * e], s_[192 * b:192 * e], sl.ctypes.data_as(ctypes.c_void_p),
                                           None, u64(rands[b:e]), e - b) == (G.SUCCESS if want else G.VERIFY_FAIL)


# ------------------------------------------------------------------ C3
def test_c3_sync_committee_fav_512x10000(G, L, F, REF, registry):
    """C3: 10,000 messages, the same 512-key committee, a seeded 1 % invalid (signed by
    the committee minus one member, or another message's signature)."""
    sks, comp = registry
    m, k = 10_000, 512
    rng = np.random.default_rng(3)
    committee = rng.choice(1 << 20, size=k, replace=False).astype(np.uint32)
    s = sum(sks[int(i)] for i in committee) % F.R_ORDER
    msgs = F.messages(m, b"c3")
    sigs = bytearray(F.sign([s] * m, msgs))
    invalid = sorted(rng.choice(m, size=m // 100, replace=False).tolist())
    for j, i in enumerate(invalid):
        if j % 2 == 0:  # signed by the committee minus one member
            sigs[192 * i:192 * i + 192] = F.sign([(s - sks[int(committee[0])]) % F.R_ORDER], msgs[32 * i:32 * i + 32])
        else:  # another message's signature
            o = (i + 1) % m
            sigs[192 * i:192 * i + 192] = sigs[192 * o:192 * o + 192] if o not in invalid else F.sign([s], b"x" * 32)
    sigs = bytes(sigs)
    idx = np.tile(committee, m)
    off = np.arange(0, k * m + 1, k, dtype=np.uint32)
    moff = G.u32_array(range(0, 32 * m + 1, 32))
    v = G.i32_array(m)
    G.check(L.gbls_fast_aggregate_verify_indexed(sigs, msgs, moff, idx.ctypes.data_as(ctypes.c_void_p),
                                                 off.ctypes.data_as(ctypes.c_void_p), m, v), "fav_indexed")
    got = [i for i in range(m) if v[i] != 0]
    assert got == invalid
    # the point-array API on a 1000-message slice, and the C oracle on a sample
    agg_pk = F.public_keys([s])
    pts = agg_pk  # one aggregate key; the batch API aggregates 512 points per message
    keys = F.public_keys([sks[int(i)] for i in committee])
    mm = 1000
    v2 = G.i32_array(mm)
    G.check(L.gbls_fast_aggregate_verify_batch(sigs[:192 * mm], msgs[:32 * mm], G.u32_array(range(0, 32 * mm + 1, 32)),
                                               keys * mm, G.u32_array(range(0, k * mm + 1, k)), mm, v2), "fav_batch")
    assert [v2[i] for i in range(mm)] == [v[i] for i in range(mm)]
    for i in list(range(0, m, 997)) + invalid[:6]:
        ref = REF.ref_verify(sigs[192 * i:192 * i + 192], msgs[32 * i:32 * i + 32], 32, pts)
        assert bool(ref) == (v[i] == 0), i


# ------------------------------------------------------------------ fused MultiVerifier::finish
def test_multi_verify_compressed_golden_and_decode_errors(G, L, F):
    """gbls_multi_verify_compressed (decompression on the device inside the multi_verify
    submission) gives every golden multi_verify verdict from the 96-byte signatures, and a
    signature that fails to decode returns its BLST_ERROR status (finish's
    Err(DecompressionFailed)) with the per-signature statuses, before any verdict."""
    from grandine_amd import bls as B
    with open(os.path.join(ROOT, "tests", "golden", "multi_verify.json")) as fh:
        cases = json.load(fh)["cases"]
    for c in cases:
        msgs = [bytes.fromhex(h) for h in c["msgs"]]
        if not msgs or any(len(m) != 32 for m in msgs):
            continue
        pks = []
        for h in c["pks"]:
            if h == "c0" + "00" * 47:
                pks.append(B.PublicKey.default())
            else:
                st, raw = B.decompress_public_keys([bytes.fromhex(h)], validate=False)[0]
                pks.append(B.PublicKey(raw))
        rc = B.Signature.multi_verify_compressed(msgs, [bytes.fromhex(h) for h in c["sigs"]], pks,
                                                 [int(r) for r in c["rands"]])
        assert (rc == G.SUCCESS) == c["expect"], c.get("note")  # undecodable: its status
    n = 64
    msgs, sigs, pks, rands = F.c2_batch(n, seed=77)
    comp = ctypes.create_string_buffer(96 * n)
    G.check(L.gbls_g2_compress(sigs, n, comp), "compress")
    st = G.i32_array(n)
    r64 = (ctypes.c_uint64 * n)(*rands)
    assert L.gbls_multi_verify_compressed(msgs, comp, pks, None, None, r64, n, st) == G.SUCCESS
    assert list(st) == [0] * n
    bad = bytearray(comp.raw)
    bad[96 * 17] &= 0x7F  # clear the compression flag: BAD_ENCODING
    rc = L.gbls_multi_verify_compressed(msgs, bytes(bad), pks, None, None, r64, n, st)
    assert rc == G.BAD_ENCODING and st[17] == G.BAD_ENCODING
    assert [s for i, s in enumerate(st) if i != 17] == [0] * (n - 1)
    swapped = bytearray(comp.raw)
    swapped[96 * 3:96 * 4], swapped[96 * 4:96 * 5] = comp.raw[96 * 4:96 * 5], comp.raw[96 * 3:96 * 4]
    assert L.gbls_multi_verify_compressed(msgs, bytes(swapped), pks, None, None, r64, n, st) == G.VERIFY_FAIL
    # exactly one key source
    assert L.gbls_multi_verify_compressed(msgs, comp, None, None, None, r64, n, st) == G.VERIFY_FAIL


def test_multi_verify_compressed_block_shape(G, L, F, registry):
    """C1 shape through the fused entry: 131 sets whose keys are registry aggregates (1, 1,
    128 x 512, 512 keys), equal to decompress + gbls_multi_verify_indexed, and rejecting a
    swapped signature pair."""
    sks, comp_keys = registry
    rng = np.random.default_rng(9)
    sizes = [1, 1] + [512] * 128 + [512]
    idx = np.concatenate([rng.choice(N_REG, size=s, replace=False) for s in sizes]).astype(np.uint32)
    off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint32)
    n = len(sizes)
    msgs = F.messages(n, b"c1-test")
    sigs, _ = F.committee_signatures(sks, idx, off, msgs)
    comp = ctypes.create_string_buffer(96 * n)
    G.check(L.gbls_g2_compress(sigs, n, comp), "compress")
    rands = (ctypes.c_uint64 * n)(*F.rands(n, 9))
    pidx, poff = idx.ctypes.data_as(ctypes.c_void_p), off.ctypes.data_as(ctypes.c_void_p)
    st = G.i32_array(n)
    assert L.gbls_multi_verify_compressed(msgs, comp, None, pidx, poff, rands, n, st) == G.SUCCESS
    assert L.gbls_multi_verify_indexed(msgs, sigs, pidx, poff, rands, n) == G.SUCCESS
    bad = bytearray(comp.raw)
    bad[96 * 40:96 * 41], bad[96 * 41:96 * 42] = comp.raw[96 * 41:96 * 42], comp.raw[96 * 40:96 * 41]
    assert L.gbls_multi_verify_compressed(msgs, bytes(bad), None, pidx, poff, rands, n, st) == G.VERIFY_FAIL
