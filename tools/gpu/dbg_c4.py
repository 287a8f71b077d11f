"""Debug: C4-shaped committees (registry indices + per-set key ranges) verified in k shards
through the partials entry point + one final exponentiation, against the verdict entry point
on the same shard.  Prints one line per (shard count, path)."""
import ctypes
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from grandine_amd import _lib as G  # noqa: E402
from grandine_amd import factory as F  # noqa: E402

dev = torch.device("cuda", 0)
L = G.lib()
nreg = 1 << 16
ncom = int(sys.argv[1]) if len(sys.argv) > 1 else 256
sks, comp = F.registry(nreg, seed=b"dbg-c4")
assert not F.load_registry(comp).any()
idx_all, off_all = F.committees(nreg - 64, ncom, seed=4)
msgs_all = F.messages(ncom, b"c4")
rands_all = F.rands(ncom, 4)


def dnp(a):
    return torch.from_numpy(np.ascontiguousarray(a).view(np.int32)).to(dev)


def ptr(t):
    return ctypes.c_void_p(t.data_ptr())


st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
for k in (1, 2, 4):
    parts = torch.zeros(k * 576, dtype=torch.uint8, device=dev)
    errs = torch.zeros(k, dtype=torch.int32, device=dev)
    shard_v = []
    for j in range(k):
        c0, c1 = ncom * j // k, ncom * (j + 1) // k
        idx = idx_all[off_all[c0]:off_all[c1]]
        off = (off_all[c0:c1 + 1] - off_all[c0]).astype(np.uint32)
        msgs = msgs_all[32 * c0:32 * c1]
        sigs, _ = F.committee_signatures(sks, idx, off, msgs)
        rands = F.rands(ncom, 4)[c0:c1]
        n = c1 - c0
        d_m = torch.frombuffer(bytearray(msgs), dtype=torch.uint8).to(dev)
        d_s = torch.frombuffer(bytearray(sigs), dtype=torch.uint8).to(dev)
        d_r = torch.tensor([x - (1 << 64) if x >= 1 << 63 else x for x in rands], dtype=torch.int64, device=dev)
        d_i, d_o = dnp(idx), dnp(off)
        seg = G.u32_array([0, n])
        v = torch.full((1,), -1, dtype=torch.int32, device=dev)
        G.check(L.gbls_multi_verify_indexed_segments_device(ptr(d_m), ptr(d_s), ptr(d_i), ptr(d_o), ptr(d_r), n, seg, 1,
                                                            ptr(v), st), "verdict")
        G.check(L.gbls_multi_verify_indexed_partials_device(ptr(d_m), ptr(d_s), ptr(d_i), ptr(d_o), ptr(d_r), n, seg, 1,
                                                            ctypes.c_void_p(parts.data_ptr() + 576 * j),
                                                            ctypes.c_void_p(errs.data_ptr() + 4 * j), st), "partial")
        torch.cuda.synchronize()
        shard_v.append(int(v.item()))
        # the same shard's partial alone
        v1 = torch.full((1,), -1, dtype=torch.int32, device=dev)
        G.check(L.gbls_final_verify_partials_device(ctypes.c_void_p(parts.data_ptr() + 576 * j),
                                                    ctypes.c_void_p(errs.data_ptr() + 4 * j), 1, 1, ptr(v1), st), "f1")
        torch.cuda.synchronize()
        print("k=%d shard %d: n=%d verdict-path %d, own-partial %d, err %d" % (k, j, n, shard_v[-1], int(v1.item()),
                                                                           int(errs[j].item())), flush=True)
    v = torch.full((1,), -1, dtype=torch.int32, device=dev)
    G.check(L.gbls_final_verify_partials_device(ptr(parts), ptr(errs), k, 1, ptr(v), st), "final")
    torch.cuda.synchronize()
    print("k=%d: combined partials verdict %d" % (k, int(v.item())), flush=True)
