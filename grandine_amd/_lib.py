"""ctypes binding of the C ABI in include/grandine_bls_gpu.h.

The shared library is built in-tree (grandine_amd/lib/libgrandine_bls.so) by
``__graft_entry__.build()`` / ``make -C grandine_amd``.  There is no CPU fallback:
if the library or a gfx950 device is missing, calls raise ``EngineUnavailable``.
"""

from __future__ import annotations

import ctypes
import os
import threading

_PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_PKG, "lib", "libgrandine_bls.so")
# Experiment builds (tools/gpu sweeps): GBLS_LIB may name another build of the library
# INSIDE this package directory (make LIB=lib_x ...); anything else is refused, so a stray
# environment variable cannot swap the verifier for an arbitrary shared object.
_override = os.environ.get("GBLS_LIB")
if _override:
    _real = os.path.realpath(_override)
    if os.path.commonpath([_real, os.path.realpath(_PKG)]) != os.path.realpath(_PKG):
        raise ImportError(f"GBLS_LIB={_override!r} is outside {_PKG}; refusing to load it")
    import sys as _sys

    print(f"grandine_amd: experiment build {_real} (GBLS_LIB)", file=_sys.stderr)
    LIB_PATH = _real

# GBLS_INIT_TUNING (include/grandine_bls_gpu.h): tests and sweeps that set the engine's
# tuning environment variables call enable_tuning() before the first lib() call.
INIT_TUNING = 0x200
INIT_PER_CHECK = 0x400  # grouped single checks off (deterministic per-check verdicts)
INIT_NO_COALESCE = 0x100  # cross-caller coalescing off
_tuning = False


def enable_tuning():
    """Let the engine read its tuning environment variables (tests / sweeps only)."""
    global _tuning
    _tuning = True

# status codes (BLST_ERROR mirror)
SUCCESS = 0
BAD_ENCODING = 1
POINT_NOT_ON_CURVE = 2
POINT_NOT_IN_GROUP = 3
AGGR_TYPE_MISMATCH = 4
VERIFY_FAIL = 5
PK_IS_INFINITY = 6
BAD_SCALAR = 7
ERR_NO_DEVICE = 100
CALL_BLOCK = 0x1  # gbls_multi_verify_compressed_ex: block-import priority class

P1_BYTES = 96
P2_BYTES = 192
FP12_BYTES = 576

EXPORTS = [
    "gbls_init",
    "gbls_set_policy",
    "gbls_last_error",
    "gbls_version",
    "gbls_device_count",
    "gbls_g1_decompress",
    "gbls_g2_decompress",
    "gbls_g2_validate",
    "gbls_g1_compress",
    "gbls_g2_compress",
    "gbls_g1_aggregate",
    "gbls_g1_aggregate_segments",
    "gbls_g2_aggregate",
    "gbls_g2_aggregate_segments",
    "gbls_registry_set",
    "gbls_registry_size",
    "gbls_g1_aggregate_indexed",
    "gbls_fast_aggregate_verify_indexed",
    "gbls_multi_verify_indexed",
    "gbls_multi_verify_compressed",
    "gbls_multi_verify_compressed_ex",
    "gbls_multi_verify_bisect",
    "gbls_multi_verify_indexed_segments_device",
    "gbls_fast_aggregate_verify_indexed_device",
    "gbls_multi_verify_indexed_partials_device",
    "gbls_verify",
    "gbls_fast_aggregate_verify",
    "gbls_aggregate_verify_batch",
    "gbls_verify_batch_compressed",
    "gbls_fast_aggregate_verify_batch",
    "gbls_multi_verify",
    "gbls_multi_verify_segments",
    "gbls_multi_verify_segments_device",
    "gbls_multi_verify_partials_device",
    "gbls_final_verify_partials_device",
    "gbls_sk_to_pk",
    "gbls_sign",
    "gbls_hash_to_g2",
    "gbls_measure_mad64_peak",
    "gbls_profile",
    "gbls_profile_read",
    "gbls_profile_reset",
    "gbls_stage_name",
]


class EngineUnavailable(RuntimeError):
    pass


_lock = threading.Lock()
_lib = None
_ready = False

_c = ctypes
_u8p = _c.c_char_p
_sz = _c.c_size_t
_vp = _c.c_void_p


def _share_torch_hip_runtime():
    """PyTorch-ROCm bundles its own libamdhip64 with the same soname as /opt/rocm's.  The
    first one loaded serves the whole process, and torch cannot enumerate devices on a
    runtime other than its own -- so when torch is installed, load it before the engine
    so both share torch's HIP runtime (the engine's device buffers are then ordinary
    torch-visible allocations and streams interoperate)."""
    try:
        import torch  # noqa: F401
    except ImportError:
        pass


def load_library():
    """Load the shared library without touching the GPU (symbol checks only)."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise EngineUnavailable(f"{LIB_PATH} not built (run __graft_entry__.build())")
            _share_torch_hip_runtime()
            lib = _c.CDLL(LIB_PATH)
            sig = {
                "gbls_init": (_c.c_int, [_c.c_uint32, _c.c_uint32]),
                "gbls_set_policy": (_c.c_uint32, [_c.c_uint32]),
                "gbls_last_error": (_c.c_int, []),
                "gbls_version": (_c.c_char_p, []),
                "gbls_device_count": (_c.c_int, []),
                "gbls_g1_decompress": (_c.c_int, [_vp, _sz, _c.c_int, _vp, _vp]),
                "gbls_g2_decompress": (_c.c_int, [_vp, _sz, _vp, _vp]),
                "gbls_g2_validate": (_c.c_int, [_vp, _sz, _vp]),
                "gbls_g1_compress": (_c.c_int, [_vp, _sz, _vp]),
                "gbls_g2_compress": (_c.c_int, [_vp, _sz, _vp]),
                "gbls_g1_aggregate": (_c.c_int, [_vp, _sz, _vp]),
                "gbls_g1_aggregate_segments": (_c.c_int, [_vp, _vp, _sz, _vp, _vp]),
                "gbls_g2_aggregate": (_c.c_int, [_vp, _sz, _vp]),
                "gbls_g2_aggregate_segments": (_c.c_int, [_vp, _vp, _sz, _vp, _vp]),
                "gbls_registry_set": (_c.c_int, [_sz, _vp, _sz, _vp]),
                "gbls_registry_size": (_sz, []),
                "gbls_g1_aggregate_indexed": (_c.c_int, [_vp, _vp, _sz, _vp, _vp]),
                "gbls_fast_aggregate_verify_indexed": (_c.c_int, [_vp, _vp, _vp, _vp, _vp, _sz, _vp]),
                "gbls_multi_verify_indexed": (_c.c_int, [_vp, _vp, _vp, _vp, _vp, _sz]),
                "gbls_multi_verify_compressed": (_c.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _sz, _vp]),
                "gbls_multi_verify_compressed_ex": (_c.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _sz, _vp,
                                                               _c.c_uint32]),
                "gbls_multi_verify_bisect": (_c.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _sz, _vp]),
                "gbls_fast_aggregate_verify_indexed_device": (_c.c_int, [_vp, _vp, _vp, _vp, _sz, _vp, _vp]),
                "gbls_multi_verify_indexed_partials_device": (
                    _c.c_int, [_vp, _vp, _vp, _vp, _vp, _sz, _vp, _sz, _vp, _vp, _vp]),
                "gbls_multi_verify_indexed_segments_device": (
                    _c.c_int, [_vp, _vp, _vp, _vp, _vp, _sz, _vp, _sz, _vp, _vp]),
                "gbls_verify": (_c.c_int, [_vp, _vp, _sz, _vp]),
                "gbls_fast_aggregate_verify": (_c.c_int, [_vp, _vp, _sz, _vp, _sz]),
                "gbls_aggregate_verify_batch": (_c.c_int, [_vp, _vp, _vp, _vp, _sz, _vp]),
                "gbls_verify_batch_compressed": (_c.c_int, [_vp, _vp, _vp, _vp, _sz, _vp, _vp]),
                "gbls_fast_aggregate_verify_batch": (_c.c_int, [_vp, _vp, _vp, _vp, _vp, _sz, _vp]),
                "gbls_multi_verify": (_c.c_int, [_vp, _vp, _vp, _vp, _sz]),
                "gbls_multi_verify_segments": (_c.c_int, [_vp, _vp, _vp, _vp, _sz, _vp, _sz, _vp]),
                "gbls_multi_verify_segments_device": (
                    _c.c_int, [_vp, _vp, _vp, _vp, _sz, _vp, _sz, _vp, _vp]),
                "gbls_multi_verify_partials_device": (
                    _c.c_int, [_vp, _vp, _vp, _vp, _sz, _vp, _sz, _vp, _vp, _vp]),
                "gbls_final_verify_partials_device": (_c.c_int, [_vp, _vp, _sz, _sz, _vp, _vp]),
                "gbls_sk_to_pk": (_c.c_int, [_vp, _sz, _vp]),
                "gbls_sign": (_c.c_int, [_vp, _vp, _vp, _sz, _vp]),
                "gbls_hash_to_g2": (_c.c_int, [_vp, _vp, _sz, _vp, _sz, _vp]),
                "gbls_measure_mad64_peak": (_c.c_double, []),
                "gbls_profile": (_c.c_int, [_c.c_int]),
                "gbls_profile_read": (_c.c_int, [_vp, _vp, _c.c_int]),
                "gbls_profile_reset": (None, []),
                "gbls_stage_name": (_c.c_char_p, [_c.c_int]),
            }
            for name, (res, args) in sig.items():
                fn = getattr(lib, name)
                fn.restype = res
                fn.argtypes = args
            _lib = lib
    return _lib


def lib(device_mask: int = 0, flags: int = 0):
    """The library with the device initialised (raises if no gfx950 device).  The first
    call's device_mask / flags configure the engine (gbls_init is idempotent)."""
    global _ready
    L = load_library()
    if not _ready:
        with _lock:
            if not _ready:
                if _tuning:
                    flags |= INIT_TUNING
                if L.gbls_init(device_mask, flags) != SUCCESS:
                    raise EngineUnavailable(
                        f"gbls_init failed (error {L.gbls_last_error()}): no usable gfx950 device")
                _ready = True
    return L


def buf(data: bytes):
    """A ctypes buffer holding ``data`` (kept alive by the caller)."""
    return _c.create_string_buffer(bytes(data), len(data) or 1)


def addr(b) -> int:
    return _c.addressof(b)


def check(rc: int, what: str):
    if rc != SUCCESS:
        raise EngineUnavailable(f"{what} failed: rc={rc} err={lib().gbls_last_error()}")


def i32_array(n: int):
    return (_c.c_int32 * max(n, 1))()


def u32_array(vals):
    vals = list(vals)
    return (_c.c_uint32 * max(len(vals), 1))(*vals)


def u64_array(vals):
    vals = list(vals)
    return (_c.c_uint64 * max(len(vals), 1))(*vals)
