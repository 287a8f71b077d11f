"""Timing of the final verdict kernel alone: gbls_final_verify_partials_device on random
Miller-value partials (verdicts irrelevant), NSEG segments, REPS launches.  Run under
rocprofv3 --kernel-trace --stats for the per-kernel average."""
import ctypes
import sys
import time

import torch

sys.path.insert(0, ".")
from grandine_amd import _lib as G  # noqa: E402

nseg = int(sys.argv[1]) if len(sys.argv) > 1 else 1
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
dev = torch.device("cuda", 0)
L = G.lib()
g = torch.Generator().manual_seed(1)
words = torch.randint(0, 1 << 31, (nseg, 12, 12), generator=g, dtype=torch.int64)
words[:, :, 11] &= 0x0fffffff  # each coefficient < 2^380 < p
parts = words.to(torch.int32).to(dev).contiguous()
errs = torch.zeros(nseg, dtype=torch.int32, device=dev)
v = torch.full((nseg,), -1, dtype=torch.int32, device=dev)
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
p = lambda t: ctypes.c_void_p(t.data_ptr())
for _ in range(3):
    G.check(L.gbls_final_verify_partials_device(p(parts), p(errs), 1, nseg, p(v), st), "final")
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(reps):
    G.check(L.gbls_final_verify_partials_device(p(parts), p(errs), 1, nseg, p(v), st), "final")
torch.cuda.synchronize()
print("nseg %d: %.1f us per call (host clock, %d calls), verdicts %s" % (
    nseg, (time.perf_counter() - t0) / reps * 1e6, reps, v[:4].tolist()), flush=True)
