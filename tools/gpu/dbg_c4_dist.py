"""Debug: bench.py's 2-rank C4 flow (one epoch split into whole committees per rank) with every
intermediate verdict printed: the rank's shard through the verdict entry point, its own partial
alone, and the gathered partials.  Run under torch.distributed.run (gloo, one GPU)."""
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch
    import torch.distributed as dist

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dist.init_process_group("gloo")
    from grandine_amd import _lib as G
    from grandine_amd import factory as F

    L = G.lib(1, 0)
    dev = torch.device("cuda", 0)
    nreg = int(sys.argv[1])
    ncom = int(sys.argv[2])
    sks, comp = F.registry(nreg, seed=b"c4-registry")
    assert not F.load_registry(comp).any()
    idx_all, off_all = F.committees(nreg - 576, ncom, seed=4)
    c0, c1 = ncom * rank // world, ncom * (rank + 1) // world
    idx = idx_all[off_all[c0]:off_all[c1]]
    off = (off_all[c0:c1 + 1] - off_all[c0]).astype(np.uint32)
    msgs = F.messages(ncom, b"c4")[32 * c0:32 * c1]
    sigs, _ = F.committee_signatures(sks, idx, off, msgs)
    rands = F.rands(ncom, 4)[c0:c1]
    n = c1 - c0

    def dnp(a):
        return torch.from_numpy(np.ascontiguousarray(a).view(np.int32)).to(dev)

    def ptr(t):
        return ctypes.c_void_p(t.data_ptr())

    d_m = torch.frombuffer(bytearray(msgs), dtype=torch.uint8).to(dev)
    d_s = torch.frombuffer(bytearray(sigs), dtype=torch.uint8).to(dev)
    d_r = torch.tensor([x - (1 << 64) if x >= 1 << 63 else x for x in rands], dtype=torch.int64, device=dev)
    d_i, d_o = dnp(idx), dnp(off)
    seg = G.u32_array([0, n])
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    v = torch.full((1,), -1, dtype=torch.int32, device=dev)
    G.check(L.gbls_multi_verify_indexed_segments_device(ptr(d_m), ptr(d_s), ptr(d_i), ptr(d_o), ptr(d_r), n, seg, 1,
                                                        ptr(v), st), "verdict")
    part = torch.zeros(576, dtype=torch.uint8, device=dev)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    G.check(L.gbls_multi_verify_indexed_partials_device(ptr(d_m), ptr(d_s), ptr(d_i), ptr(d_o), ptr(d_r), n, seg, 1,
                                                        ptr(part), ptr(err), st), "partial")
    v1 = torch.full((1,), -1, dtype=torch.int32, device=dev)
    G.check(L.gbls_final_verify_partials_device(ptr(part), ptr(err), 1, 1, ptr(v1), st), "own")
    torch.cuda.synchronize()
    parts = [torch.empty(576, dtype=torch.uint8) for _ in range(world)]
    errs = [torch.empty(1, dtype=torch.int32) for _ in range(world)]
    dist.all_gather(parts, part.cpu())
    dist.all_gather(errs, err.cpu())
    dparts, derrs = torch.cat(parts).to(dev), torch.cat(errs).to(dev)
    vg = torch.full((1,), -1, dtype=torch.int32, device=dev)
    G.check(L.gbls_final_verify_partials_device(ptr(dparts), ptr(derrs), world, 1, ptr(vg), st), "final")
    torch.cuda.synchronize()
    out = [None] * world
    dist.all_gather_object(out, {"rank": rank, "n": n, "verdict": int(v.item()), "own_partial": int(v1.item()),
                                 "err": int(err.item()), "gathered": int(vg.item()),
                                 "idx0": int(idx[0]), "off_last": int(off[-1])})
    if rank == 0:
        print(json.dumps({"world": world, "ranks": out}), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
