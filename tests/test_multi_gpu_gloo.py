"""CPU, world_size 2 (gloo): the multi-GPU flow of bench.py and INTEGRATION.md section 3,
run with the C oracle (oracle/bls_ref.c) standing in for each GPU's shard.

Each rank takes a contiguous slice of the sets and computes its Miller partial
F_g = prod ML(r_i pk_i, H(m_i)) * ML(-g1, S_g) plus an error flag. The ranks all-gather
(576-byte Fp12, flag). Rank 0 multiplies the partials and runs one final
exponentiation. The verdict must equal the fixture's unsharded
verdict for every golden multi_verify case.
"""
import ctypes
import json
import os
import socket
import subprocess
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
LIB = os.path.join(ROOT, "oracle", "_build", "libbls_ref.so")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _cases():
    import sys
    sys.path.insert(0, ROOT)
    from oracle import bls12_381 as O

    mont = 1 << 384

    def fp_b(x):
        return (x * mont % O.P).to_bytes(48, "little")

    with open(os.path.join(GOLD, "multi_verify.json")) as fh:
        cases = json.load(fh)["cases"]
    out = []
    for c in cases:
        sigs, pks = [], []
        for h in c["sigs"]:
            p = O.g2_decompress(bytes.fromhex(h))[1]
            sigs.append(bytes(192) if p is None else fp_b(p[0][0]) + fp_b(p[0][1]) + fp_b(p[1][0]) + fp_b(p[1][1]))
        for h in c["pks"]:
            p = O.g1_decompress(bytes.fromhex(h))[1]
            pks.append(bytes(96) if p is None else fp_b(p[0]) + fp_b(p[1]))
        out.append({"msgs": [bytes.fromhex(h) for h in c["msgs"]], "sigs": sigs, "pks": pks,
                    "rands": [int(r) for r in c["rands"]], "expect": c["expect"], "note": c["note"]})
    return out


def _worker(rank, world, port, result_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    C = ctypes.CDLL(LIB)
    C.ref_multi_verify_partial.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p,
                                           ctypes.POINTER(ctypes.c_uint64), ctypes.c_size_t, ctypes.c_char_p]
    C.ref_final_verify_partials.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_int32), ctypes.c_size_t]
    verdicts = []
    for c in _cases():
        n = len(c["msgs"])
        b, e = n * rank // world, n * (rank + 1) // world  # contiguous shard, as bench.py
        part = ctypes.create_string_buffer(576)
        rands = (ctypes.c_uint64 * max(1, e - b))(*c["rands"][b:e])
        err = C.ref_multi_verify_partial(b"".join(c["msgs"][b:e]), b"".join(c["sigs"][b:e]),
                                         b"".join(c["pks"][b:e]), rands, e - b, part)
        mine = torch.frombuffer(bytearray(part.raw), dtype=torch.uint8)
        parts = [torch.empty(576, dtype=torch.uint8) for _ in range(world)]
        dist.all_gather(parts, mine)
        errs = [torch.zeros(1, dtype=torch.int32) for _ in range(world)]
        dist.all_gather(errs, torch.tensor([err], dtype=torch.int32))
        if rank == 0:
            blob = b"".join(bytes(p.numpy().tobytes()) for p in parts)
            ev = (ctypes.c_int32 * world)(*[int(x.item()) for x in errs])
            verdicts.append({"note": c["note"], "expect": c["expect"],
                             "got": bool(C.ref_final_verify_partials(blob, ev, world))})
    dist.barrier()
    dist.destroy_process_group()
    if rank == 0:
        with open(result_path, "w") as fh:
            json.dump(verdicts, fh)


@pytest.fixture(scope="module")
def oracle_lib():
    subprocess.check_call(["make", "-C", os.path.join(ROOT, "oracle"), "-s"])
    return LIB


def test_sharded_multi_verify_world2(oracle_lib):
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "verdicts.json")
        mp.spawn(_worker, args=(2, _free_port(), path), nprocs=2, join=True)
        with open(path) as fh:
            res = json.load(fh)
    assert len(res) >= 6
    for r in res:
        assert r["got"] == r["expect"], r["note"]


def test_partials_compose_across_shard_counts(oracle_lib):
    """Splitting a valid batch into 1, 2 or 3 shards gives the same verdict; a tampered
    shard partial (one bit of one Fp coefficient) breaks it."""
    C = ctypes.CDLL(LIB)
    C.ref_multi_verify_partial.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p,
                                           ctypes.POINTER(ctypes.c_uint64), ctypes.c_size_t, ctypes.c_char_p]
    C.ref_final_verify_partials.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_int32), ctypes.c_size_t]
    c = next(x for x in _cases() if x["expect"] and len(x["msgs"]) >= 6)
    n = len(c["msgs"])
    for k in (1, 2, 3):
        parts = []
        for g in range(k):
            b, e = n * g // k, n * (g + 1) // k
            buf = ctypes.create_string_buffer(576)
            rands = (ctypes.c_uint64 * (e - b))(*c["rands"][b:e])
            assert C.ref_multi_verify_partial(b"".join(c["msgs"][b:e]), b"".join(c["sigs"][b:e]),
                                              b"".join(c["pks"][b:e]), rands, e - b, buf) == 0
            parts.append(buf.raw)
        errs = (ctypes.c_int32 * k)(*([0] * k))
        assert C.ref_final_verify_partials(b"".join(parts), errs, k) == 1
        bad = bytearray(parts[-1])
        bad[0] ^= 1
        assert C.ref_final_verify_partials(b"".join(parts[:-1]) + bytes(bad), errs, k) == 0
