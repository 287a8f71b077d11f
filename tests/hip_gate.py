"""A host-released gate for GPU streams (GPU test helper): a stream that waits on the gate
(hipStreamWaitValue32 on a pinned host word) runs none of its later work until the host opens
it.  Tests use it to hold verifications queued on a stream while another call must complete,
so they assert ORDER (this call returned / finished while that stream was provably still
blocked) instead of wall-clock overlap.

Always open the gate in a `finally` (or use `with Gate() as g:`): a stream left waiting would
keep its work queued.  The runtime is torch's libamdhip64 (the one the engine shares, see
grandine_amd/_lib.py)."""
import ctypes
import os


def _hip():
    import torch
    path = os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so")
    hip = ctypes.CDLL(path)  # already loaded by torch: the same handle
    hip.hipHostMalloc.restype = ctypes.c_int
    hip.hipHostMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
    hip.hipHostFree.restype = ctypes.c_int
    hip.hipHostFree.argtypes = [ctypes.c_void_p]
    hip.hipStreamWaitValue32.restype = ctypes.c_int
    hip.hipStreamWaitValue32.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint,
                                         ctypes.c_uint32]
    return hip


class Gate:
    WAIT_GTE = 0x0  # hipStreamWaitValueGte

    def __init__(self):
        self.hip = _hip()
        self.word = ctypes.c_void_p()
        rc = self.hip.hipHostMalloc(ctypes.byref(self.word), 64, 0)
        if rc != 0:
            raise RuntimeError(f"hipHostMalloc failed ({rc})")
        ctypes.memset(self.word, 0, 64)
        self.open = False

    def hold(self, stream_handle: int):
        """Every later operation on the stream waits until open()."""
        rc = self.hip.hipStreamWaitValue32(ctypes.c_void_p(stream_handle), self.word, 1, self.WAIT_GTE,
                                           0xFFFFFFFF)
        if rc != 0:
            raise RuntimeError(f"hipStreamWaitValue32 failed ({rc})")

    def release(self):
        ctypes.c_uint32.from_address(self.word.value).value = 1
        self.open = True

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.release()
        return False
