"""The C1 bench's gossip load alone: 16 threads each submitting 64-set gbls_multi_verify
calls (host pointers) for SECONDS; prints sets/s and the per-call latency spread.  Under
rocprofv3 --kernel-trace, tools/prof/merge_sizes.py then reads how the coalescer merged."""
import ctypes
import sys
import threading
import time

sys.path.insert(0, ".")
from grandine_amd import _lib as G  # noqa: E402
from grandine_amd import factory as F  # noqa: E402

secs = float(sys.argv[1]) if len(sys.argv) > 1 else 3.0
nthr = int(sys.argv[2]) if len(sys.argv) > 2 else 16
if "--tuning" in sys.argv:  # GBLS_MERGE_TARGET / GBLS_LEADERS / ... sweeps
    G.enable_tuning()
L = G.lib()
gm, gs, gp, gr = F.c2_batch(64, seed=64)
r64 = (ctypes.c_uint64 * 64)(*gr)
for _ in range(5):
    assert L.gbls_multi_verify(gm, gs, gp, r64, 64) == G.SUCCESS
stop = threading.Event()
lat = []
errs = []


def worker():
    while not stop.is_set():
        t = time.perf_counter()
        if L.gbls_multi_verify(gm, gs, gp, r64, 64) != G.SUCCESS:
            errs.append(1)
        lat.append(time.perf_counter() - t)


ths = [threading.Thread(target=worker) for _ in range(nthr)]
t0 = time.perf_counter()
for x in ths:
    x.start()
time.sleep(secs)
stop.set()
for x in ths:
    x.join()
el = time.perf_counter() - t0
assert not errs
lat.sort()
print("threads %d: %d calls in %.2f s = %.0f sets/s; latency p50 %.2f ms p90 %.2f ms max %.2f ms" % (
    nthr, len(lat), el, len(lat) * 64 / el, lat[len(lat) // 2] * 1e3, lat[int(len(lat) * 0.9)] * 1e3, lat[-1] * 1e3),
    flush=True)
