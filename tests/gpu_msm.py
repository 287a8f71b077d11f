"""Subprocess of tests/test_gpu_paths.py: the engine with GBLS_MSM_MIN=1, so every
single-segment multi_verify computes S = sum r_i sig_i by the bucket MSM (k_msm.hip)
instead of per-set scalar multiplication.  Runs the golden multi_verify cases, edge
cases (infinite signatures, zero scalar, equal scalars) and a 4096-set batch against
the C oracle; prints one JSON line."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["GBLS_MSM_MIN"] = "1"

from grandine_amd import _lib as G  # noqa: E402
G.enable_tuning()  # the engine reads the knob set above
from grandine_amd import bls as B  # noqa: E402
from grandine_amd import factory as F  # noqa: E402


def u64(v):
    return (ctypes.c_uint64 * len(v))(*v)


def main():
    L = G.lib()
    C = ctypes.CDLL(os.path.join(ROOT, "oracle", "_build", "libbls_ref.so"))
    C.ref_multi_verify.argtypes = [ctypes.c_char_p] * 3 + [ctypes.POINTER(ctypes.c_uint64), ctypes.c_size_t,
                                                           ctypes.c_int]
    res = {"golden": [], "c2": []}
    with open(os.path.join(ROOT, "tests", "golden", "multi_verify.json")) as fh:
        cases = json.load(fh)["cases"]
    for c in cases:
        msgs = [bytes.fromhex(h) for h in c["msgs"]]
        sigs = [B.Signature.try_from(bytes.fromhex(h)) for h in c["sigs"]]
        pks = []
        for h in c["pks"]:
            if h == "c0" + "00" * 47:
                pks.append(B.PublicKey.default())
            else:
                st, raw = B.decompress_public_keys([bytes.fromhex(h)], validate=False)[0]
                pks.append(B.PublicKey(raw))
        got = B.Signature.multi_verify(msgs, sigs, pks, [int(r) for r in c["rands"]])
        res["golden"].append(got == c["expect"])
    n = 4096
    msgs, sigs, pks, rands = F.c2_batch(n, seed=31)
    variants = [("valid", msgs, sigs, rands)]
    bad = bytearray(sigs)
    bad[192 * 77:192 * 78] = sigs[192 * 78:192 * 79]
    variants.append(("swapped", msgs, bytes(bad), rands))
    inf = bytearray(sigs)
    inf[192 * 9:192 * 10] = bytes(192)
    variants.append(("infinite sig", msgs, bytes(inf), rands))
    same = list(rands)
    same[100:200] = [same[100]] * 100  # many equal scalars: crowded buckets
    variants.append(("equal scalars", msgs, sigs, same))
    small = [(i % 7) + 1 for i in range(n)]  # tiny scalars: most digits zero
    variants.append(("small scalars", msgs, sigs, small))
    for name, m, s, r in variants:
        gpu = L.gbls_multi_verify(m, s, pks, u64(r), n) == G.SUCCESS
        ref = bool(C.ref_multi_verify(m, s, pks, u64(r), n, 16))
        res["c2"].append([name, gpu, ref])
    # several segments at once (per-segment buckets): the 2nd and 4th corrupted
    m2, s2, p2, r2 = F.c2_batch(3000, seed=32)
    off = [0, 500, 1300, 1301, 2100, 3000]
    mb = bytearray(m2)
    mb[32 * 700] ^= 1
    mb[32 * 1500] ^= 1
    vs = G.i32_array(5)
    G.check(L.gbls_multi_verify_segments(bytes(mb), s2, p2, u64(r2), 3000, G.u32_array(off), 5, vs), "segs")
    res["segments"] = [vs[i] for i in range(5)]
    zero = list(rands)
    zero[5] = 0
    v = G.i32_array(1)
    G.check(L.gbls_multi_verify_segments(msgs, sigs, pks, u64(zero), n, G.u32_array([0, n]), 1, v), "segs")
    res["zero_scalar"] = v[0]
    print(json.dumps(res))


if __name__ == "__main__":
    main()
