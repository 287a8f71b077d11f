"""Subprocess of tests/test_gpu_dropin.py (its own engine, GBLS_TRACE_STALLS=1): a context's
first call, which grows every workspace, must not wait for another stream's work (VERDICT r05
"next 1": a fresh context's growth synchronised the caller's stream, 18-24 ms host stalls in the
C4 timed loop, gbls_capi.hip Ctx::ensure before r06).

* stream A warms its context, then is HELD by a host-released gate (tests/hip_gate.py) and gets
  a 4096-set verification queued behind the gate;
* on a new stream B a 8192-set verification leases a context that has never run (created by
  gbls_init, or new) -- every buffer grows, the staging ring is sized -- and B is then
  synchronised;
* B's call must return AND complete while the gate still holds A (A provably busy), with the
  right verdict; then A is released and its verdict checked.
A watchdog opens the gate after 60 s, so a host wait inside B's call fails the test instead of
hanging it.  Prints one JSON line."""
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
    L = G.lib(0, 1)
    dev = torch.device("cuda", 0)
    t = lambda b: torch.frombuffer(bytearray(b), dtype=torch.uint8).to(dev)
    batches = {}
    for n, seed in ((4096, 31), (8192, 32)):
        msgs, sigs, pks, rands = F.c2_batch(n, seed=seed)
        r = torch.from_numpy(np.array(rands, dtype=np.uint64).view(np.int64)).to(dev)
        batches[n] = (t(msgs), t(sigs), t(pks), r)
    verdicts = torch.full((3,), -1, dtype=torch.int32, device=dev)

    def run(n, stream, slot):
        m, s, p, r = batches[n]
        with torch.cuda.stream(stream):
            return L.gbls_multi_verify_segments_device(
                m.data_ptr(), s.data_ptr(), p.data_ptr(), r.data_ptr(), n, G.u32_array([0, n]), 1,
                verdicts[slot:].data_ptr(), ctypes.c_void_p(stream.cuda_stream))

    A, B = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    G.check(run(4096, A, 0), "warm A")
    torch.cuda.synchronize()
    verdicts.fill_(-1)
    torch.cuda.synchronize()
    out = {}

    def fresh_call():
        t0 = time.perf_counter()
        out["rc_b"] = run(8192, B, 1)
        out["enqueue_ms"] = round(1e3 * (time.perf_counter() - t0), 3)
        B.synchronize()  # B's kernels must run although A is held
        out["done_ms"] = round(1e3 * (time.perf_counter() - t0), 3)

    gate = Gate()
    try:
        gate.hold(A.cuda_stream)
        out["rc_a"] = run(4096, A, 0)  # queued behind the gate
        worker = threading.Thread(target=fresh_call, daemon=True)
        worker.start()
        worker.join(timeout=60)
        finished_while_held = not worker.is_alive()
        a_busy = not A.query()
        v_b = verdicts[1].item() if finished_while_held else None
    finally:
        gate.release()
    worker.join(timeout=120)
    torch.cuda.synchronize()
    res = {"rc_a": out.get("rc_a"), "rc_b": out.get("rc_b"), "finished_while_held": finished_while_held,
           "a_busy_while_held": a_busy, "v_b_while_held": v_b, "verdicts": verdicts.cpu().tolist()[:2],
           "enqueue_ms": out.get("enqueue_ms"), "done_ms": out.get("done_ms")}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
