"""Minimal HIP device-memory helpers for tests (ctypes on libamdhip64).

libffmi.so is loaded first, so this resolves to the same HIP runtime.
"""
import ctypes
import os

import numpy as np

import flexflow_amd.ffmi as F

_hip = None


def hip():
    global _hip
    if _hip is None:
        F.lib()  # make sure libffmi (and its HIP runtime) is loaded first
        path = "/opt/rocm/lib/libamdhip64.so"
        if not os.path.exists(path):
            path = "libamdhip64.so"
        H = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
        H.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
        H.hipFree.argtypes = [ctypes.c_void_p]
        H.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        H.hipMemset.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t]
        H.hipDeviceSynchronize.argtypes = []
        H.hipGetDeviceCount.argtypes = [ctypes.POINTER(ctypes.c_int)]
        H.hipStreamCreate.argtypes = [ctypes.POINTER(ctypes.c_void_p)]
        H.hipStreamSynchronize.argtypes = [ctypes.c_void_p]
        H.hipEventCreate.argtypes = [ctypes.POINTER(ctypes.c_void_p)]
        H.hipEventRecord.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        H.hipEventSynchronize.argtypes = [ctypes.c_void_p]
        H.hipEventElapsedTime.argtypes = [ctypes.POINTER(ctypes.c_float), ctypes.c_void_p,
                                          ctypes.c_void_p]
        _hip = H
    return _hip


def device_count():
    n = ctypes.c_int(0)
    try:
        if hip().hipGetDeviceCount(ctypes.byref(n)) != 0:
            return 0
    except OSError:
        return 0
    return n.value


def sync():
    assert hip().hipDeviceSynchronize() == 0


class Buf:
    """A device buffer holding a numpy array's bytes."""

    def __init__(self, arr=None, nbytes=None, dtype=None, shape=None):
        if arr is not None:
            arr = np.ascontiguousarray(arr)
            nbytes, dtype, shape = arr.nbytes, arr.dtype, arr.shape
        self.nbytes, self.dtype, self.shape = int(nbytes), np.dtype(dtype), tuple(shape)
        self.ptr = ctypes.c_void_p()
        assert hip().hipMalloc(ctypes.byref(self.ptr), max(self.nbytes, 16)) == 0
        if arr is not None:
            assert hip().hipMemcpy(self.ptr, arr.ctypes.data, self.nbytes, 1) == 0
        else:
            assert hip().hipMemset(self.ptr, 0, max(self.nbytes, 16)) == 0

    @classmethod
    def empty(cls, shape, dtype):
        dtype = np.dtype(dtype)
        n = int(np.prod(shape)) * dtype.itemsize
        return cls(nbytes=n, dtype=dtype, shape=shape)

    def get(self):
        out = np.empty(self.shape, self.dtype)
        sync()
        assert hip().hipMemcpy(out.ctypes.data, self.ptr, self.nbytes, 2) == 0
        return out

    def __del__(self):
        if getattr(self, "ptr", None) and self.ptr.value:
            hip().hipFree(self.ptr)
            self.ptr = None


class Timer:
    def __init__(self, stream=None):
        self.stream = stream
        self.a, self.b = ctypes.c_void_p(), ctypes.c_void_p()
        hip().hipEventCreate(ctypes.byref(self.a))
        hip().hipEventCreate(ctypes.byref(self.b))

    def start(self):
        hip().hipEventRecord(self.a, self.stream)

    def stop(self):
        hip().hipEventRecord(self.b, self.stream)
        hip().hipEventSynchronize(self.b)
        ms = ctypes.c_float()
        hip().hipEventElapsedTime(ctypes.byref(ms), self.a, self.b)
        return ms.value


def f16(x):
    return np.asarray(x, np.float32).astype(np.float16)


def ulp_diff(a16, b16):
    """distance in fp16 ulps (monotonic int mapping)."""
    def key(x):
        u = np.asarray(x, np.float16).view(np.uint16).astype(np.int32)
        return np.where(u & 0x8000, 0x8000 - (u & 0x7FFF), u + 0x8000)
    return np.abs(key(a16) - key(b16))


def report(name, **kv):
    """Append one measured parity figure to gpurun_out/parity_report.jsonl
    (read back after a GPU run; DESIGN.md quotes it)."""
    import json
    import os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    os.makedirs(os.path.join(root, "gpurun_out"), exist_ok=True)
    with open(os.path.join(root, "gpurun_out", "parity_report.jsonl"), "a") as f:
        f.write(json.dumps(dict(test=name, **kv)) + "\n")
