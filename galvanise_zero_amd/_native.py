"""ctypes bindings of the in-tree native libraries (include/gzero_nn.h, include/gzero_engine.h).

The product path has no fallback: if a library is missing or fails to load, the call raises.
Libraries live in galvanise_zero_amd/lib/ (built by galvanise_zero_amd/csrc/Makefile).
"""

import ctypes
import os

import numpy as np

LIB_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib")
GZ_MAX_ROLES = 4

_libs = {}


class NativeLibraryMissing(RuntimeError):
    pass


def lib_path(name):
    return os.path.join(LIB_DIR, name)


def _load(name):
    lib = _libs.get(name)
    if lib is None:
        path = lib_path(name)
        if not os.path.exists(path):
            raise NativeLibraryMissing("native library %s not built (run __graft_entry__.build() or "
                                       "make -C galvanise_zero_amd/csrc)" % path)
        lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
        _libs[name] = lib
    return lib


###############################################################################
# libgz_nn.so

class GzNetDesc(ctypes.Structure):
    _fields_ = [("input_channels", ctypes.c_int),
                ("input_columns", ctypes.c_int),
                ("input_rows", ctypes.c_int),
                ("cnn_filter_size", ctypes.c_int),
                ("cnn_kernel_size", ctypes.c_int),
                ("residual_layers", ctypes.c_int),
                ("role_count", ctypes.c_int),
                ("policy_dist_count", ctypes.c_int * GZ_MAX_ROLES),
                ("value_hidden_size", ctypes.c_int),
                ("num_values", ctypes.c_int),
                ("leaky_relu", ctypes.c_int),
                ("flatten_nchw", ctypes.c_int)]


_FP = ctypes.POINTER(ctypes.c_float)


def nn_lib():
    lib = _load("libgz_nn.so")
    if not getattr(lib, "_gz_typed", False):
        lib.gz_net_create.restype = ctypes.c_void_p
        lib.gz_net_create.argtypes = [ctypes.POINTER(GzNetDesc), ctypes.c_int]
        lib.gz_net_destroy.argtypes = [ctypes.c_void_p]
        lib.gz_net_weight_count.restype = ctypes.c_size_t
        lib.gz_net_weight_count.argtypes = [ctypes.c_void_p]
        lib.gz_net_set_weights.argtypes = [ctypes.c_void_p, _FP, ctypes.c_size_t]
        lib.gz_net_set_weights_device.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
        lib.gz_net_forward.argtypes = [ctypes.c_void_p, _FP, ctypes.c_int,
                                       ctypes.POINTER(_FP), _FP]
        lib.gz_net_forward_device.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                              ctypes.c_int, ctypes.POINTER(ctypes.c_void_p),
                                              ctypes.c_void_p]
        lib.gz_net_last_kernel_ms.restype = ctypes.c_float
        lib.gz_net_last_kernel_ms.argtypes = [ctypes.c_void_p]
        lib.gz_net_flops_per_eval.restype = ctypes.c_double
        lib.gz_net_flops_per_eval.argtypes = [ctypes.c_void_p]
        lib.gz_nn_last_error.restype = ctypes.c_char_p
        lib._gz_typed = True
    return lib


def make_net_desc(desc):
    d = GzNetDesc()
    d.input_channels = desc.input_channels
    d.input_columns = desc.input_columns
    d.input_rows = desc.input_rows
    d.cnn_filter_size = desc.cnn_filter_size
    d.cnn_kernel_size = desc.cnn_kernel_size
    d.residual_layers = desc.residual_layers
    d.role_count = len(desc.policy_dist_count)
    for i, p in enumerate(desc.policy_dist_count):
        d.policy_dist_count[i] = p
    d.value_hidden_size = desc.value_hidden_size
    d.num_values = desc.num_values
    d.leaky_relu = int(desc.leaky_relu)
    d.flatten_nchw = int(desc.flatten_nchw)
    return d


def _fptr(a):
    return a.ctypes.data_as(_FP)


class HipNet(object):
    """Owner of a gz_net handle: the MI355X forward of one network on one device."""

    def __init__(self, desc, device=0):
        self.lib = nn_lib()
        self.desc = desc
        self._cdesc = make_net_desc(desc)
        self.handle = self.lib.gz_net_create(ctypes.byref(self._cdesc), device)
        if not self.handle:
            raise RuntimeError("gz_net_create failed: %s" % self.lib.gz_nn_last_error().decode())
        self.weight_count = self.lib.gz_net_weight_count(self.handle)

    def _check(self, rc, what):
        if rc != 0:
            raise RuntimeError("%s failed: %s" % (what, self.lib.gz_nn_last_error().decode()))

    def set_weights(self, blob):
        blob = np.ascontiguousarray(blob, dtype=np.float32)
        if blob.size != self.weight_count:
            raise ValueError("weight blob has %d floats, network expects %d" % (blob.size, self.weight_count))
        self._check(self.lib.gz_net_set_weights(self.handle, _fptr(blob), blob.size), "gz_net_set_weights")

    def set_weights_device(self, ptr, count):
        self._check(self.lib.gz_net_set_weights_device(self.handle, ctypes.c_void_p(ptr), count),
                    "gz_net_set_weights_device")

    def forward(self, planes):
        d = self.desc
        planes = np.ascontiguousarray(planes, dtype=np.float32)
        n = planes.shape[0]
        assert planes.size == n * d.input_channels * d.input_columns * d.input_rows
        pols = [np.empty((n, p), dtype=np.float32) for p in d.policy_dist_count]
        val = np.empty((n, d.num_values), dtype=np.float32)
        arr = (_FP * len(pols))(*[_fptr(p) for p in pols])
        self._check(self.lib.gz_net_forward(self.handle, _fptr(planes), n, arr, _fptr(val)),
                    "gz_net_forward")
        return pols + [val]

    def forward_device(self, stream, d_planes, n, d_policies, d_values):
        arr = (ctypes.c_void_p * len(d_policies))(*d_policies)
        self._check(self.lib.gz_net_forward_device(self.handle, ctypes.c_void_p(stream),
                                                   ctypes.c_void_p(d_planes), n, arr,
                                                   ctypes.c_void_p(d_values)),
                    "gz_net_forward_device")

    def last_kernel_ms(self):
        return self.lib.gz_net_last_kernel_ms(self.handle)

    def flops_per_eval(self):
        return self.lib.gz_net_flops_per_eval(self.handle)

    def close(self):
        if self.handle:
            self.lib.gz_net_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
