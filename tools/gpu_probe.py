"""Quick on-device probe: mad64 peak, and per-stage timing of one multi_verify batch."""
import ctypes, hashlib, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from grandine_amd import _lib as G

L = G.lib()
print("version", L.gbls_version().decode())
t = time.time(); pk = L.gbls_measure_mad64_peak(); print("mad64 peak %.3e /s (%.1fs)" % (pk, time.time() - t))
n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
sks = b"".join((int.from_bytes(hashlib.sha256(b"sk%d" % i).digest(), "big") % R).to_bytes(32, "big") for i in range(n))
msgs = b"".join(hashlib.sha256(b"m%d" % i).digest() for i in range(n))
pks = ctypes.create_string_buffer(96 * n); sigs = ctypes.create_string_buffer(192 * n)
off = G.u32_array(range(0, 32 * n + 1, 32))
t = time.time(); G.check(L.gbls_sk_to_pk(sks, n, pks), "sk_to_pk"); print("sk_to_pk %d: %.3fs" % (n, time.time() - t))
t = time.time(); G.check(L.gbls_sign(sks, msgs, off, n, sigs), "sign"); print("sign %d: %.3fs" % (n, time.time() - t))
rands = G.u64_array([(i * 0x9E3779B97F4A7C15 + 1) & ((1 << 64) - 1) or 1 for i in range(n)])
for it in range(3):
    t = time.time(); v = L.gbls_multi_verify(msgs, sigs, pks, rands, n); dt = time.time() - t
    print("multi_verify n=%d verdict=%d %.3fs -> %.0f sets/s" % (n, v, dt, n / dt))
bad = bytearray(msgs); bad[5] ^= 1
print("multi_verify corrupted verdict", L.gbls_multi_verify(bytes(bad), sigs, pks, rands, n))
