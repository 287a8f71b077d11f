"""Timing of the hash_to_G2 map stage alone at C1's shape: gbls_hash_to_g2 on N messages
(REPS calls); run under rocprofv3 --kernel-trace --stats for the per-kernel averages."""
import ctypes
import sys

sys.path.insert(0, ".")
from grandine_amd import _lib as G  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 131
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 30
L = G.lib()
msgs = bytes(range(256)) * ((32 * n) // 256 + 1)
msgs = msgs[:32 * n]
off = G.u32_array([32 * i for i in range(n + 1)])
out = (ctypes.c_uint8 * (192 * n))()
for _ in range(reps):
    G.check(L.gbls_hash_to_g2(msgs, off, n, None, 0, out), "hash_to_g2")
print("ok", n, reps)
