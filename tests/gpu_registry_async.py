"""Subprocess of tests/test_gpu_dropin.py (its own engine, so the registry it grows is not the
one the other GPU tests share): gbls_registry_set with GROWTH while registry-indexed
verifications are still running on a device stream (VERDICT r04 "next 5").

* two indexed multi_verify submissions of 131072 sets each (~30 ms of GPU work apiece) are
  queued on two torch streams (gbls_multi_verify_indexed_segments_device: asynchronous, reading
  the registry), the second with one swapped signature;
* the two streams are HELD by a host-released gate (tests/hip_gate.py: hipStreamWaitValue32 on
  a pinned word) before the submissions are queued, so none of their work can run until the
  host opens it; registry_set then loads keys far past the table's capacity (the table is
  reallocated and the old one retired behind those readers on the GPU) and must RETURN while the
  gate is still closed -- any device-wide synchronisation or host wait for those readers would
  block it (a watchdog opens the gate after 60 s and the test fails): ordering, not wall-clock;
* every queued verdict must be right (the readers kept a valid table), and afterwards sets over
  the old slots and over the new slice verify (the loaded entries were carried over).
Also replicas (gbls_init flags & 0xff = 2): the same growth on two engines of the one GPU.
Prints one JSON line."""
import ctypes
import json
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from grandine_amd import _lib as G  # noqa: E402
from grandine_amd import factory as F  # noqa: E402
from hip_gate import Gate  # noqa: E402  (tests/, the script's own directory)


def main():
    import torch
    replicas = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    L = G.lib(0, replicas)
    dev = torch.device("cuda", 0)
    n_reg, n, k, nst = 4096, 131072, 2, 2
    sks, comp = F.registry(n_reg, seed=b"async")
    assert not F.load_registry(comp).any()
    cap0 = L.gbls_registry_size()
    idx = [(7 * i) % n_reg for i in range(n)]
    msgs = F.messages(n, b"async")
    sigs = F.sign([sks[i] for i in idx], msgs)
    bad = bytearray(sigs)
    bad[192 * 100:192 * 101] = sigs[192 * 101:192 * 102]
    t = lambda b: torch.frombuffer(bytearray(b), dtype=torch.uint8).to(dev)
    d_msgs, d_sigs, d_bad = t(msgs), t(sigs), t(bytes(bad))
    d_idx = torch.tensor(idx, dtype=torch.int32, device=dev)
    d_r = torch.from_numpy(np.array(F.rands(n, 3), dtype=np.uint64).view(np.int64)).to(dev)
    verdicts = torch.full((k,), -1, dtype=torch.int32, device=dev)
    off = G.u32_array([0, n])
    streams = [torch.cuda.Stream(dev) for _ in range(nst)]
    # warm-up (every stream's context sized), then the timed queue
    for s in streams:
        with torch.cuda.stream(s):
            G.check(L.gbls_multi_verify_indexed_segments_device(
                d_msgs.data_ptr(), d_sigs.data_ptr(), d_idx.data_ptr(), None, d_r.data_ptr(), n, off, 1,
                verdicts.data_ptr(), ctypes.c_void_p(s.cuda_stream)), "warm")
    torch.cuda.synchronize()
    new_sks, new_comp = F.registry(64, seed=b"async-new")
    verdicts.fill_(-1)
    torch.cuda.synchronize()
    first = 400_000
    st = (ctypes.c_int32 * 64)()
    out = {}

    def queue_and_set():
        t_q = time.perf_counter()
        for j in range(k):
            s = streams[j % nst]
            with torch.cuda.stream(s):
                G.check(L.gbls_multi_verify_indexed_segments_device(
                    d_msgs.data_ptr(), (d_bad if j % 3 == 1 else d_sigs).data_ptr(), d_idx.data_ptr(), None,
                    d_r.data_ptr(), n, off, 1, verdicts[j:].data_ptr(), ctypes.c_void_p(s.cuda_stream)), "queued")
        out["enqueue_ms"] = round(1e3 * (time.perf_counter() - t_q), 3)
        # growth while the readers are held: 64 new keys at index 400000 (the table holds ~5k)
        t0 = time.perf_counter()
        out["rc"] = L.gbls_registry_set(first, G.buf(new_comp), 64, st)
        out["set_ms"] = round(1e3 * (time.perf_counter() - t0), 3)

    gate = Gate()
    try:
        for s in streams:
            gate.hold(s.cuda_stream)
        worker = threading.Thread(target=queue_and_set, daemon=True)
        worker.start()
        worker.join(timeout=60)
        returned_while_held = not worker.is_alive()
        held_busy = all(not s.query() for s in streams)  # the gate still holds every reader
    finally:
        gate.release()
    worker.join(timeout=120)
    torch.cuda.synchronize()
    res = {"rc": out.get("rc"), "statuses": sorted(set(st)), "returned_while_held": returned_while_held,
           "held_busy": held_busy, "enqueue_ms": out.get("enqueue_ms"), "set_ms": out.get("set_ms"),
           "verdicts": verdicts.cpu().tolist(), "size": L.gbls_registry_size(), "cap0": cap0,
           "replicas": L.gbls_device_count()}
    # old slots and the new slice both resolve after the growth
    m2 = F.messages(128, b"async-2")
    i2 = [(13 * i) % n_reg for i in range(64)] + [first + i for i in range(64)]
    s2 = F.sign([sks[i] for i in i2[:64]] + new_sks, m2)
    res["after"] = L.gbls_multi_verify_indexed(m2, s2, G.u32_array(i2), None,
                                               (ctypes.c_uint64 * 128)(*F.rands(128, 4)), 128)
    res["gap"] = L.gbls_multi_verify_indexed(m2[:32], s2[:192], G.u32_array([first - 1]), None,
                                             (ctypes.c_uint64 * 1)(5), 1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
