"""Debug probe: cross-check GPU and C-oracle Miller partials under both final exps."""
import ctypes, os, sys, json
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch
from grandine_amd import _lib as G, factory as F
C = ctypes.CDLL(os.path.join(ROOT, "oracle", "_build", "libbls_ref.so"))
C.ref_multi_verify_partial.argtypes = [ctypes.c_char_p]*3 + [ctypes.POINTER(ctypes.c_uint64), ctypes.c_size_t, ctypes.c_char_p]
C.ref_final_verify_partials.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_int32), ctypes.c_size_t]
L = G.lib()
dev = torch.device("cuda", 0)
n = 64; h = 32
msgs, sigs, pks, rands = F.c2_batch(n, seed=13)
def u64(v): return (ctypes.c_uint64 * len(v))(*v)
def cpart(b, e):
    out = ctypes.create_string_buffer(576)
    assert C.ref_multi_verify_partial(msgs[32*b:32*e], sigs[192*b:192*e], pks[96*b:96*e], u64(rands[b:e]), e-b, out) == 0
    return out.raw
def gpart(b, e):
    d = lambda x: torch.frombuffer(bytearray(x), dtype=torch.uint8).to(dev)
    m, s, p = d(msgs[32*b:32*e]), d(sigs[192*b:192*e]), d(pks[96*b:96*e])
    r = torch.tensor([x - (1 << 64) if x >= 1 << 63 else x for x in rands[b:e]], dtype=torch.int64, device=dev)
    out = torch.zeros(576, dtype=torch.uint8, device=dev); err = torch.zeros(1, dtype=torch.int32, device=dev)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    assert L.gbls_multi_verify_partials_device(m.data_ptr(), s.data_ptr(), p.data_ptr(), r.data_ptr(), e-b, G.u32_array([0, e-b]), 1, out.data_ptr(), err.data_ptr(), st) == 0
    torch.cuda.synchronize()
    return bytes(out.cpu().numpy().tobytes())
def gfinal(parts):
    t = torch.frombuffer(bytearray(b"".join(parts)), dtype=torch.uint8).to(dev)
    errs = torch.zeros(len(parts), dtype=torch.int32, device=dev); v = torch.full((1,), -1, dtype=torch.int32, device=dev)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    assert L.gbls_final_verify_partials_device(t.data_ptr(), errs.data_ptr(), len(parts), 1, v.data_ptr(), st) == 0
    torch.cuda.synchronize(); return int(v.item())
def cfinal(parts):
    ev = (ctypes.c_int32 * len(parts))(*([0]*len(parts)))
    return C.ref_final_verify_partials(b"".join(parts), ev, len(parts))
GA, GB, CA, CB = gpart(0, h), gpart(h, n), cpart(0, h), cpart(h, n)
res = {}
for name, parts in [("GA", [GA]), ("GB", [GB]), ("CA", [CA]), ("CB", [CB]), ("GA.GB", [GA, GB]), ("CA.CB", [CA, CB]), ("GA.CB", [GA, CB]), ("CA.GB", [CA, GB])]:
    res[name] = {"gpu_final": gfinal(parts), "c_final_ok": cfinal(parts)}
res["GA==CA"] = GA == CA
res["GA_head"] = GA[:16].hex(); res["CA_head"] = CA[:16].hex()
print(json.dumps(res))
