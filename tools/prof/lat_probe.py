#!/usr/bin/env python3
"""Latency probe for rocprofv3 kernel traces: serial host-pointer calls of one small shape
(gossip: 64 single-key sets via gbls_multi_verify; block: the C1 131-set fused finish over
a registry).  Usage: python tools/prof/lat_probe.py {gossip|block} [calls]"""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402

from grandine_amd import _lib as G  # noqa: E402
from grandine_amd import factory as F  # noqa: E402

kind = sys.argv[1] if len(sys.argv) > 1 else "gossip"
calls = int(sys.argv[2]) if len(sys.argv) > 2 else 30
L = G.lib()
if kind == "gossip":
    n = int(os.environ.get("PROBE_N", "64"))
    gm, gs, gp, gr = F.c2_batch(n, seed=64)
    r = (ctypes.c_uint64 * n)(*gr)

    def call():
        return L.gbls_multi_verify(gm, gs, gp, r, n)
else:
    nreg = 1 << 17
    sks, comp = F.registry(nreg, seed=b"probe-registry")
    assert not F.load_registry(comp).any()
    rng = np.random.default_rng(1)
    sizes = [1, 1] + [512] * 128 + [512]
    idx = np.concatenate([rng.choice(nreg, size=s, replace=False) for s in sizes]).astype(np.uint32)
    off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint32)
    n = len(sizes)
    msgs = F.messages(n, b"c1")
    sigs, _ = F.committee_signatures(sks, idx, off, msgs)
    comp_sigs = ctypes.create_string_buffer(96 * n)
    G.check(L.gbls_g2_compress(sigs, n, comp_sigs), "compress")
    r = (ctypes.c_uint64 * n)(*F.rands(n, 1))
    pidx, poff = idx.ctypes.data_as(ctypes.c_void_p), off.ctypes.data_as(ctypes.c_void_p)
    st = G.i32_array(n)

    def call():
        return L.gbls_multi_verify_compressed(msgs, comp_sigs, None, pidx, poff, r, n, st)
lat = []
for _ in range(calls):
    t = time.perf_counter()
    assert call() == G.SUCCESS
    lat.append(time.perf_counter() - t)
lat.sort()
print("%s n=%d calls=%d p50 %.3f ms min %.3f ms" % (kind, n, calls, lat[len(lat) // 2] * 1e3, lat[0] * 1e3))
