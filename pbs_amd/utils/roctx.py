"""roctx ranges from Python: gang epochs and bench policy
windows appear on a ``rocprofv3 --marker-trace`` timeline next to the tenant
kernels and the native scheduler ranges (csrc/hip/runtime.cpp).  No-ops when
the HIP library is not loaded (CPU-only runs)."""
from __future__ import annotations

import contextlib


def _lib():
    from .. import _native as N
    return N._hip


@contextlib.contextmanager
def range(name: str):
    lib = _lib()
    if lib is None:
        yield
        return
    lib.gpbs_roctx_push(name.encode())
    try:
        yield
    finally:
        lib.gpbs_roctx_pop()


def mark(name: str):
    lib = _lib()
    if lib is not None:
        lib.gpbs_roctx_mark(name.encode())
