"""Helpers shared by the -m gpu tests (no tests here)."""
import ctypes

import numpy as np


class Pinned(object):
    """hipHostMalloc'd buffer (what the runner's pools use), viewed as a float32 numpy array."""

    def __init__(self, n):
        self.hip = ctypes.CDLL("libamdhip64.so.7")   # the runtime torch / libgz_nn.so already loaded
        self.hip.hipHostMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
        self.hip.hipHostFree.argtypes = [ctypes.c_void_p]
        self.ptr = ctypes.c_void_p()
        assert self.hip.hipHostMalloc(ctypes.byref(self.ptr), max(1, n) * 4, 0) == 0
        self.a = np.ctypeslib.as_array(ctypes.cast(self.ptr, ctypes.POINTER(ctypes.c_float)), shape=(max(1, n),))[:n]

    def free(self):
        if self.ptr:
            self.hip.hipHostFree(self.ptr)
            self.ptr = None


def err(a, b):
    d = np.abs(a.astype(np.float64) - b.astype(np.float64))
    return float(d.max()), float(d.mean())


def kl(ref, got):
    r = np.clip(ref.astype(np.float64), 1e-30, None)
    g = np.clip(got.astype(np.float64), 1e-30, None)
    return float((r * np.log(r / g)).sum(axis=1).max())
