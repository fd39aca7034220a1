"""roctx ranges / marks for rocprofv3 (``--marker-trace``) and a round-window timer.

SURVEY 5.1: the reference has no tracing at all.  Here every federation phase
(consensus, W0 broadcast, the round loop, checkpoints, result export) is a roctx
range, so a ``rocprofv3 --kernel-trace --marker-trace`` timeline shows the HIP
kernels of each round under their phase.  The ranges call the ROCm roctx
library through ctypes (librocprofiler-sdk-roctx, or the legacy libroctx64);
without it, or with ``GFEDNTM_ROCTX=0``, they are no-ops.
"""
from __future__ import annotations

import contextlib
import ctypes
import os
import time
from typing import Optional

_lib = None
_tried = False


def _roctx():
    global _lib, _tried
    if not _tried:
        _tried = True
        if os.environ.get("GFEDNTM_ROCTX", "1") != "0":
            for name in ("librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so",
                         "libroctx64.so.4", "libroctx64.so"):
                for path in (name, os.path.join("/opt/rocm/lib", name)):
                    try:
                        lib = ctypes.CDLL(path)
                        lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                        lib.roctxRangePushA.restype = ctypes.c_int
                        lib.roctxRangePop.restype = ctypes.c_int
                        lib.roctxMarkA.argtypes = [ctypes.c_char_p]
                        _lib = lib
                        return _lib
                    except (OSError, AttributeError):
                        continue
    return _lib


def available() -> bool:
    return _roctx() is not None


@contextlib.contextmanager
def trace_range(name: str):
    lib = _roctx()
    if lib is not None:
        lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        if lib is not None:
            lib.roctxRangePop()


def mark(name: str) -> None:
    lib = _roctx()
    if lib is not None:
        lib.roctxMarkA(name.encode())


class RoundWindow:
    """Host wall time and documents over a window of rounds (device-synchronised at
    the window end only, so the round loop stays asynchronous)."""

    def __init__(self, sync=None):
        self.sync = sync
        self.reset()

    def reset(self):
        self.t0 = time.perf_counter()
        self.rounds = 0
        self.docs = 0

    def add(self, docs: int):
        self.rounds += 1
        self.docs += int(docs)

    def close(self) -> Optional[dict]:
        if self.rounds == 0:
            return None
        if self.sync is not None:
            self.sync()
        dt = time.perf_counter() - self.t0
        out = {"rounds": self.rounds, "docs": self.docs, "wall_s": dt,
               "ms_per_round": 1e3 * dt / self.rounds, "docs_per_s": self.docs / dt if dt else None}
        self.reset()
        return out
