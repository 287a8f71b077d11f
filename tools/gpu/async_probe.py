"""How asynchronous are the device entry points?  Times each gbls_multi_verify_indexed_segments_device
enqueue (8 calls over 1, 2 or 4 torch streams) against the GPU time of the work; prints one line per
configuration.  usage: python tools/gpu/async_probe.py"""
import ctypes
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from grandine_amd import _lib as G  # noqa: E402
from grandine_amd import factory as F  # noqa: E402


def main():
    import torch
    L = G.lib()
    dev = torch.device("cuda", 0)
    n_reg, n = 4096, 16384
    sks, comp = F.registry(n_reg, seed=b"async")
    assert not F.load_registry(comp).any()
    idx = [(7 * i) % n_reg for i in range(n)]
    msgs = F.messages(n, b"async")
    sigs = F.sign([sks[i] for i in idx], msgs)
    t = lambda b: torch.frombuffer(bytearray(b), dtype=torch.uint8).to(dev)
    d_msgs, d_sigs = t(msgs), t(sigs)
    d_idx = torch.tensor(idx, dtype=torch.int32, device=dev)
    d_r = torch.from_numpy(np.array(F.rands(n, 3), dtype=np.uint64).view(np.int64)).to(dev)
    verdicts = torch.full((16,), -1, dtype=torch.int32, device=dev)
    off = G.u32_array([0, n])
    for nst in (1, 2, 4):
        streams = [torch.cuda.Stream(dev) for _ in range(nst)]
        for rep in range(2):  # first pass sizes every context
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            per = []
            for j in range(8):
                s = streams[j % nst]
                a = time.perf_counter()
                with torch.cuda.stream(s):
                    G.check(L.gbls_multi_verify_indexed_segments_device(
                        d_msgs.data_ptr(), d_sigs.data_ptr(), d_idx.data_ptr(), None, d_r.data_ptr(), n, off, 1,
                        verdicts[j:].data_ptr(), ctypes.c_void_p(s.cuda_stream)), "call")
                per.append(round(1e3 * (time.perf_counter() - a), 2))
            enq = time.perf_counter() - t0
            torch.cuda.synchronize()
            tot = time.perf_counter() - t0
            print("streams=%d pass=%d enqueue_ms=%.2f total_ms=%.2f per_call_ms=%s" % (nst, rep, 1e3 * enq, 1e3 * tot, per),
                  flush=True)


if __name__ == "__main__":
    main()
