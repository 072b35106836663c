"""Kernel timing events without a system-scope fence.

torch.cuda.Event(enable_timing=True) records a HIP event whose release fence writes the GPU's dirty
caches back at every record: bracketing each launch of a training step with such pairs cost about
0.7 ms per instrumented config-2 step (bench.py, 20 vs 100 timed steps with three instrumented).  The
events here are created with hipEventDisableSystemFence: the same timestamps between the same
launches on one stream, no cache write-back.  They time only; nothing reads data across them.

API as the subset of torch.cuda.Event the engine / trainer / bench use: Event().record() on the
current stream, a.elapsed_time(b) in milliseconds (after the stream has been synchronized)."""
from __future__ import annotations

import ctypes
import os

import torch

_HIP_EVENT_DISABLE_SYSTEM_FENCE = 0x20000000
_hip = None


def _lib():
    """The HIP runtime torch loaded (the same instance that owns torch's streams)."""
    global _hip
    if _hip is None:
        path = os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so")
        lib = ctypes.CDLL(path if os.path.exists(path) else "libamdhip64.so")
        lib.hipEventCreateWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint]
        lib.hipEventRecord.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        lib.hipEventElapsedTime.argtypes = [ctypes.POINTER(ctypes.c_float), ctypes.c_void_p, ctypes.c_void_p]
        lib.hipEventDestroy.argtypes = [ctypes.c_void_p]
        for f in (lib.hipEventCreateWithFlags, lib.hipEventRecord, lib.hipEventElapsedTime, lib.hipEventDestroy):
            f.restype = ctypes.c_int
        _hip = lib
    return _hip


def _check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{what} failed: hipError {rc}")


class Event:
    __slots__ = ("_e",)

    def __init__(self):
        e = ctypes.c_void_p()
        _check(_lib().hipEventCreateWithFlags(ctypes.byref(e), _HIP_EVENT_DISABLE_SYSTEM_FENCE),
               "hipEventCreateWithFlags")
        self._e = e

    def record(self, stream: torch.cuda.Stream | None = None) -> None:
        s = stream if stream is not None else torch.cuda.current_stream()
        _check(_lib().hipEventRecord(self._e, ctypes.c_void_p(s.cuda_stream)), "hipEventRecord")

    def elapsed_time(self, end: "Event") -> float:
        ms = ctypes.c_float()
        _check(_lib().hipEventElapsedTime(ctypes.byref(ms), self._e, end._e), "hipEventElapsedTime")
        return float(ms.value)

    def __del__(self):
        if self._e is not None and _hip is not None:
            _hip.hipEventDestroy(self._e)
            self._e = None
