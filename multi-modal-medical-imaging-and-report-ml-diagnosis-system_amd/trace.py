"""roctx ranges around the phases of the train step (SURVEY §5 tracing row: the reference has
only `print`s, TP:861-862 / 922 / 1064).

`rng("mmdx/image_fwd")` is a context manager that pushes a roctx range on entry and pops it
on exit, on the calling host thread.  Under `rocprofv3 --marker-trace --kernel-trace` the
ranges appear beside the kernels, so a trace shows which phase issued which launches and
whether the RCCL kernels of `mmdx/allreduce` overlap the trunk backward.  The library is
rocprofiler-sdk's roctx (`librocprofiler-sdk-roctx.so`, the one rocprofv3's marker trace
reads; the legacy `libroctx64.so` otherwise).  Ranges cost one ctypes call each (~10 per
step); MMDX_ROCTX=0 turns them off, and without a roctx library they are no-ops (tracing is
instrumentation, not compute: nothing on the compute path depends on it).
"""
from __future__ import annotations

import contextlib
import ctypes
import os

_LIB = None
_TRIED = False


def _lib():
    global _LIB, _TRIED
    if _TRIED:
        return _LIB
    _TRIED = True
    if os.environ.get("MMDX_ROCTX", "1") == "0":
        return None
    root = os.environ.get("ROCM_PATH", "/opt/rocm")
    for name in ("librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so",
                 "libroctx64.so.4", "libroctx64.so"):
        for path in (os.path.join(root, "lib", name), name):
            try:
                lib = ctypes.CDLL(path)
            except OSError:
                continue
            lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
            lib.roctxRangePushA.restype = ctypes.c_int
            lib.roctxRangePop.argtypes = []
            lib.roctxRangePop.restype = ctypes.c_int
            _LIB = lib
            return _LIB
    return None


def available() -> bool:
    return _lib() is not None


def push(name: str) -> None:
    lib = _lib()
    if lib is not None:
        lib.roctxRangePushA(name.encode())


def pop() -> None:
    lib = _lib()
    if lib is not None:
        lib.roctxRangePop()


@contextlib.contextmanager
def rng(name: str):
    lib = _lib()
    if lib is None:
        yield
        return
    lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        lib.roctxRangePop()
