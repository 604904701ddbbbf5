"""Minimal HIP runtime plumbing over ctypes: device buffers, copies, sync.

Single-process runs (``bench.py`` at N=1, tools) use this instead of torch so
the process holds exactly one ROCm runtime -- the libamdhip64 /
libhsa-runtime64 that libopenr_spf.so links (/opt/rocm).  torch ships its own
copies; under rocprofv3, which preloads /opt/rocm's HSA runtime, a torch
process ends up with two HSA runtimes and torch's HIP teardown faults inside
the profiler's one at exit.  Multi-rank runs still use torch
for torch.distributed (RCCL).
"""

from __future__ import annotations

import ctypes as C

import numpy as np

from . import _native  # noqa: F401  -- loads libopenr_spf.so and with it its HIP runtime

_lib = C.CDLL("libamdhip64.so.7")
_lib.hipMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t]
_lib.hipFree.argtypes = [C.c_void_p]
_lib.hipMemset.argtypes = [C.c_void_p, C.c_int, C.c_size_t]
_lib.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
_lib.hipSetDevice.argtypes = [C.c_int]
_lib.hipGetErrorString.restype = C.c_char_p
_D2H, _H2D = 2, 1


def _check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{what}: {_lib.hipGetErrorString(rc).decode()}")


def set_device(i: int) -> None:
    _check(_lib.hipSetDevice(i), "hipSetDevice")


def synchronize() -> None:
    _check(_lib.hipDeviceSynchronize(), "hipDeviceSynchronize")


def device_reset() -> None:
    """Release every device resource of this process now (hipDeviceReset)."""
    _check(_lib.hipDeviceReset(), "hipDeviceReset")


class DeviceArray:
    """A device allocation of `n` elements of `dtype` (no torch)."""

    def __init__(self, n: int, dtype=np.int32, zero: bool = False) -> None:
        self.dtype = np.dtype(dtype)
        self.n = int(n)
        p = C.c_void_p()
        _check(_lib.hipMalloc(C.byref(p), max(1, self.n) * self.dtype.itemsize), "hipMalloc")
        self.ptr = int(p.value)
        if zero:
            self.zero()

    @property
    def nbytes(self) -> int:
        return self.n * self.dtype.itemsize

    def zero(self) -> None:
        """Zero the buffer and wait for it: hipMemset runs on the null stream,
        which the engine's non-blocking streams do not wait for (an unfinished
        memset overwrote a plan's first next-hop bitmaps once)."""
        _check(_lib.hipMemset(C.c_void_p(self.ptr), 0, max(1, self.nbytes)), "hipMemset")
        synchronize()

    def numpy(self) -> np.ndarray:
        out = np.empty(self.n, self.dtype)
        if self.n:
            _check(_lib.hipMemcpy(out.ctypes.data_as(C.c_void_p), C.c_void_p(self.ptr),
                                  self.nbytes, _D2H), "hipMemcpy D2H")
        return out

    def upload(self, a: np.ndarray) -> None:
        a = np.ascontiguousarray(a, self.dtype)
        _check(_lib.hipMemcpy(C.c_void_p(self.ptr), a.ctypes.data_as(C.c_void_p),
                              min(a.nbytes, self.nbytes), _H2D), "hipMemcpy H2D")

    def free(self) -> None:
        if getattr(self, "ptr", 0):
            _lib.hipFree(C.c_void_p(self.ptr))
            self.ptr = 0

    def __del__(self) -> None:
        try:
            self.free()
        except Exception:  # noqa: BLE001  -- interpreter shutdown
            pass
