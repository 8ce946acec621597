"""Device buffers for GPU tests through the C ABI's plain-pointer helpers (no torch)."""
import ctypes as C

import numpy as np

from dsocr._lib import check, lib


class Dev:
    def __init__(self, arr=None, nbytes=None, dtype=np.float32, shape=None):
        self.ptr = C.c_void_p()
        if arr is not None:
            arr = np.ascontiguousarray(arr)
            self.dtype, self.shape, nbytes = arr.dtype, arr.shape, arr.nbytes
        else:
            self.dtype, self.shape = np.dtype(dtype), shape
        check(lib().dsocr_dev_alloc(max(int(nbytes), 16), C.byref(self.ptr)))
        self.nbytes = int(nbytes)
        if arr is not None and arr.nbytes:
            check(lib().dsocr_memcpy_h2d(self.ptr, arr.ctypes.data_as(C.c_void_p), arr.nbytes))

    @classmethod
    def zeros(cls, shape, dtype=np.float32):
        return cls(np.zeros(shape, dtype))

    def get(self):
        out = np.empty(self.shape, self.dtype)
        if out.nbytes:
            check(lib().dsocr_memcpy_d2h(out.ctypes.data_as(C.c_void_p), self.ptr, out.nbytes))
        return out

    def __del__(self):
        try:
            if self.ptr:
                lib().dsocr_dev_free(self.ptr)
        except Exception:
            pass


def bf16_round(x):
    u = np.ascontiguousarray(x, np.float32).view(np.uint32).astype(np.uint64)
    u = (u + 0x7FFF + ((u >> 16) & 1)) >> 16
    return u.astype(np.uint16)


def bf16_to_f32(b):
    return (b.astype(np.uint32) << 16).view(np.float32)


def f16_bits(x):
    return np.ascontiguousarray(x, np.float32).astype(np.float16).view(np.uint16)
