"""Subprocess of tests/test_gpu_paths.py: the engine with the kernel-variant knobs given as
NAME=VALUE arguments (GBLS_ML_DMA=1, GBLS_ML_R28=0, GBLS_LANE_R28=0: the non-default forms
an operator can select), read through GBLS_INIT_TUNING.  Runs the golden multi_verify cases
and 4096-set batches (valid, swapped signature, infinite signature) plus a 4-segment batch
through the C2 path (bucket MSM, grouped Miller products) against the C oracle; prints one
JSON line."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
for kv in sys.argv[1:]:
    k, v = kv.split("=", 1)
    assert k.startswith("GBLS_"), kv
    os.environ[k] = v

from grandine_amd import _lib as G  # noqa: E402
G.enable_tuning()  # the engine reads the knobs set above
from grandine_amd import bls as B  # noqa: E402
from grandine_amd import factory as F  # noqa: E402


def u64(v):
    return (ctypes.c_uint64 * len(v))(*v)


def main():
    L = G.lib()
    C = ctypes.CDLL(os.path.join(ROOT, "oracle", "_build", "libbls_ref.so"))
    C.ref_multi_verify.argtypes = [ctypes.c_char_p] * 3 + [ctypes.POINTER(ctypes.c_uint64), ctypes.c_size_t,
                                                           ctypes.c_int]
    res = {"knobs": sys.argv[1:], "golden": [], "c2": []}
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
    msgs, sigs, pks, rands = F.c2_batch(n, seed=41)
    bad = bytearray(sigs)
    bad[192 * 300:192 * 301] = sigs[192 * 301:192 * 302]
    inf = bytearray(sigs)
    inf[192 * 17:192 * 18] = bytes(192)
    for name, s in (("valid", sigs), ("swapped", bytes(bad)), ("infinite sig", bytes(inf))):
        gpu = L.gbls_multi_verify(msgs, s, pks, u64(rands), n) == G.SUCCESS
        ref = bool(C.ref_multi_verify(msgs, s, pks, u64(rands), n, 16))
        res["c2"].append([name, gpu, ref])
    off = [0, 1024, 2048, 3072, 4096]
    mb = bytearray(msgs)
    mb[32 * 2500] ^= 1
    vs = G.i32_array(4)
    G.check(L.gbls_multi_verify_segments(bytes(mb), sigs, pks, u64(rands), n, G.u32_array(off), 4, vs), "segs")
    res["segments"] = [vs[i] for i in range(4)]
    print(json.dumps(res))


if __name__ == "__main__":
    main()
