"""Subprocess of tests/test_gpu_paths.py: the engine with a 16 MB line-coefficient budget
(GBLS_LINE_BUDGET_MB=16), so a 4096-set batch's Miller lines are made and consumed in
event slices (the running points kept in HBM between slices, gbls_capi.hip
pipeline_partials) -- the path large submissions (above the default 4 GB budget) take.
Runs a single 4096-set batch and a 4-segment batch (valid, one swapped signature in
segment 2) and prints one JSON line with the verdicts and the C oracle's."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["GBLS_LINE_BUDGET_MB"] = "16"

from grandine_amd import _lib as G  # noqa: E402
G.enable_tuning()  # the engine reads the knob set above
from grandine_amd import factory as F  # noqa: E402


def u64(v):
    return (ctypes.c_uint64 * len(v))(*v)


def main():
    L = G.lib()
    C = ctypes.CDLL(os.path.join(ROOT, "oracle", "_build", "libbls_ref.so"))
    C.ref_multi_verify.argtypes = [ctypes.c_char_p] * 3 + [ctypes.POINTER(ctypes.c_uint64), ctypes.c_size_t,
                                                           ctypes.c_int]
    n = 4096
    msgs, sigs, pks, rands = F.c2_batch(n, seed=41)
    bad = bytearray(sigs)
    bad[192 * 2100:192 * 2101] = sigs[192 * 2101:192 * 2102]  # sets 2100 and 2101 swap: segment 2
    bad[192 * 2101:192 * 2102] = sigs[192 * 2100:192 * 2101]
    bad = bytes(bad)
    res = {"single": [], "ref": [], "segments": []}
    for s in (sigs, bad):
        res["single"].append(L.gbls_multi_verify(msgs, s, pks, u64(rands), n))
        res["ref"].append(int(C.ref_multi_verify(msgs, s, pks, u64(rands), n, 16)))
    seg = G.u32_array([0, 1024, 2048, 3072, 4096])
    for s in (sigs, bad):
        v = (ctypes.c_int32 * 4)()
        rc = L.gbls_multi_verify_segments(msgs, s, pks, u64(rands), n, seg, 4, v)
        res["segments"].append([rc] + list(v))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
