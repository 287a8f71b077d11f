"""Subprocess of tests/test_gpu_paths.py: the engine with 3 engines on the one GPU
(gbls_init flags = 3), so that host calls take the multi-device paths of
gbls_capi.hip (per-engine Miller partials of one batch + one final exponentiation;
segments spread over the engines; the registry replicated per engine).  Prints one
JSON line of verdicts."""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from grandine_amd import _lib as G  # noqa: E402
from grandine_amd import factory as F  # noqa: E402


def u64(v):
    return (ctypes.c_uint64 * len(v))(*v)


def main():
    L = G.lib(0, 3)
    res = {"engines": L.gbls_device_count()}
    n = 4096
    msgs, sigs, pks, rands = F.c2_batch(n, seed=21)
    res["big_valid"] = L.gbls_multi_verify(msgs, sigs, pks, u64(rands), n)
    bad = bytearray(sigs)
    bad[192 * 4000:192 * 4001] = sigs[192 * 10:192 * 11]
    res["big_bad"] = L.gbls_multi_verify(msgs, bytes(bad), pks, u64(rands), n)
    # 6 segments, the 2nd and 5th corrupted
    m2, s2, p2, r2 = F.c2_batch(4200, seed=22)
    off = [700 * i for i in range(7)]
    mb = bytearray(m2)
    mb[32 * 800] ^= 1
    mb[32 * 3100] ^= 1
    v = G.i32_array(6)
    G.check(L.gbls_multi_verify_segments(bytes(mb), s2, p2, u64(r2), 4200, G.u32_array(off), 6, v), "segs")
    res["segs"] = [v[i] for i in range(6)]
    mb = bytearray(msgs)
    mb[32 * 7] ^= 1
    mb[32 * 3000] ^= 1
    vb = G.i32_array(n)
    G.check(L.gbls_multi_verify_bisect(bytes(mb), sigs, pks, None, None, u64(rands), n, vb), "bisect")
    res["bisect"] = [i for i in range(n) if vb[i] != 0]
    sks, comp = F.registry(100, seed=b"rep")
    assert not F.load_registry(comp).any()
    idx = [i % 100 for i in range(3000)]
    mm = F.messages(3000, b"rep")
    ss = F.sign([sks[i] for i in idx], mm)
    res["registry"] = L.gbls_multi_verify_indexed(mm, ss, G.u32_array(idx), None, u64(F.rands(3000, 9)), 3000)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
