"""Child process of tests/test_gpu_dist.py, launched by torch.distributed.run with 2 ranks on
one GPU (GBLS_BENCH_ONE_DEVICE's rehearsal: gloo instead of RCCL, which refuses two ranks on
one device).  bench.py's N-rank flow: every rank
verifies its contiguous shard of one batch into a Miller partial + error flag on the GPU
(gbls_multi_verify_partials_device), the ranks all-gather the 576-byte partials, and every
rank runs the final exponentiation over the gathered partials
(gbls_final_verify_partials_device).  Phase 1 is the clean batch; in phase 2 rank 1 flips one
message bit of its shard, and every rank must then reject.  Rank 0 prints one JSON line."""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


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
    n = 2048
    msgs, sigs, pks, rands = F.c2_batch(n, seed=77)
    b, e = n * rank // world, n * (rank + 1) // world
    k = e - b

    def verdict(m):
        dm = torch.frombuffer(bytearray(m[32 * b:32 * e]), dtype=torch.uint8).to(dev)
        ds = torch.frombuffer(bytearray(sigs[192 * b:192 * e]), dtype=torch.uint8).to(dev)
        dp = torch.frombuffer(bytearray(pks[96 * b:96 * e]), dtype=torch.uint8).to(dev)
        dr = torch.tensor([x - (1 << 64) if x >= 1 << 63 else x for x in rands[b:e]], dtype=torch.int64,
                          device=dev)
        part = torch.zeros(576, dtype=torch.uint8, device=dev)
        err = torch.zeros(1, dtype=torch.int32, device=dev)
        st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        G.check(L.gbls_multi_verify_partials_device(dm.data_ptr(), ds.data_ptr(), dp.data_ptr(), dr.data_ptr(), k,
                                                    G.u32_array([0, k]), 1, part.data_ptr(), err.data_ptr(), st),
                "partials")
        torch.cuda.current_stream().synchronize()
        parts = [torch.empty(576, dtype=torch.uint8) for _ in range(world)]
        errs = [torch.empty(1, dtype=torch.int32) for _ in range(world)]
        dist.all_gather(parts, part.cpu())
        dist.all_gather(errs, err.cpu())
        dparts = torch.cat(parts).to(dev)
        derrs = torch.cat(errs).to(dev)
        v = torch.full((1,), -1, dtype=torch.int32, device=dev)
        G.check(L.gbls_final_verify_partials_device(dparts.data_ptr(), derrs.data_ptr(), world, 1, v.data_ptr(), st),
                "final")
        return int(v.cpu()[0])

    clean = verdict(msgs)
    bad = bytearray(msgs)
    if rank == 1:
        bad[32 * (b + 17) + 3] ^= 0x40
    corrupt = verdict(bytes(bad))
    out = [None] * world
    dist.all_gather_object(out, {"rank": rank, "clean": clean, "corrupt": corrupt})
    if rank == 0:
        print(json.dumps({"world": world, "ranks": out}))
    dist.destroy_process_group()
    ok = clean == G.SUCCESS and corrupt == G.VERIFY_FAIL
    sys.exit(0 if ok else 3)


if __name__ == "__main__":
    main()
