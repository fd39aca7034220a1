"""Cross-rank digest of the shared state: failure detection of the FedAvg data plane.

After every round's FedAvg all ranks must hold the same shared state bit for bit: the
reference server pushes ONE average to every client (src/federation/server.py:477-521),
and here every chunk of the sum is computed by exactly one rank (csrc/comm.hip two-shot
kernel; RCCL's rings likewise reduce each chunk once).  A data-plane defect that returns
normally -- a stale peer cache line, a lost L2 write-back, a broken IPC mapping -- would
instead leave the replicas silently diverged.  The round loop (federation/runner.py)
therefore compares a digest of every rank's shared prefix every ``GFEDNTM_DIGEST_EVERY``
rounds (default: the error-word poll interval) and at every aligned round, and stops all
ranks with ``CommError`` on a mismatch.

The digest is ``sum_i mix(i << 32 | bits(x_i)) mod 2**64`` with splitmix64's finaliser as
``mix``: position-sensitive (a moved or flipped word changes it) and order-independent (a
sum mod 2^64), so the device kernel (csrc/comm.hip ``gfk_digest_part`` / ``_fold``) and
:func:`digest_numpy` agree bit for bit however the work is cut.  On a GPU the two kernels
run on the stream behind the round and the 8-byte result is copied to pinned memory, so
the round loop never synchronises for it (:class:`DigestProbe`).
"""
from __future__ import annotations

import ctypes as C
from typing import List, Optional, Sequence

import numpy as np
import torch

_M1, _M2, _M3 = np.uint64(0x9E3779B97F4A7C15), np.uint64(0xBF58476D1CE4E5B9), \
    np.uint64(0x94D049BB133111EB)


def digest_numpy(words: np.ndarray, chunk: int = 1 << 22) -> int:
    """The digest of a float32 / uint32 / int32 array (its 32-bit patterns, flattened)."""
    w = np.ascontiguousarray(words).reshape(-1).view(np.uint32)
    tot = np.uint64(0)
    with np.errstate(over="ignore"):
        for a in range(0, w.size, chunk):
            x = w[a:a + chunk].astype(np.uint64)
            z = (np.arange(a, a + x.size, dtype=np.uint64) << np.uint64(32)) | x
            z = z + _M1
            z = (z ^ (z >> np.uint64(30))) * _M2
            z = (z ^ (z >> np.uint64(27))) * _M3
            z = z ^ (z >> np.uint64(31))
            tot = tot + z.sum(dtype=np.uint64)
    return int(tot)


def _declare(lib):
    if getattr(lib, "_gfk_digest_declared", False):
        return
    lib.gfk_digest_launch.argtypes = [C.c_void_p, C.c_int64, C.c_void_p, C.c_int, C.c_void_p,
                                      C.c_void_p, C.c_void_p]
    lib._gfk_digest_declared = True


class DigestProbe:
    """Digests of a fixed list of buffers, taken asynchronously behind the enqueued work.

    ``take(round)`` enqueues the digests of every buffer on the current stream (device
    buffers: two kernels each + an 8-byte copy to pinned memory; host buffers: computed
    at once) and remembers the round; ``result()`` waits for the copies of the last take
    (one interval old when the runner asks, so normally already landed) and returns
    ``(round, [digest per buffer])`` or None when nothing is pending."""

    def __init__(self, buffers: Sequence[torch.Tensor]):
        self.buffers = list(buffers)
        self.device = self.buffers[0].device
        self._pending = None
        if self.device.type == "cuda":
            from ..ops import native
            self.lib = native.kernels()
            _declare(self.lib)
            cu = torch.cuda.get_device_properties(self.device).multi_processor_count
            n = max(b.numel() for b in self.buffers)
            self.nblk = int(max(1, min(4 * cu, -(-n // 4096))))
            self._part = torch.zeros(self.nblk, dtype=torch.int64, device=self.device)
            self._out = torch.zeros(len(self.buffers), dtype=torch.int64, device=self.device)
            self._host = torch.zeros(len(self.buffers), dtype=torch.int64, pin_memory=True)
            self._ev = torch.cuda.Event()
            for b in self.buffers:
                if b.dtype not in (torch.float32, torch.int32) or not b.is_contiguous() \
                        or b.data_ptr() % 16:
                    raise ValueError("digest buffers: 32-bit, contiguous, 16-byte aligned")

    def take(self, rnd: int):
        if self.device.type != "cuda":
            self._pending = (int(rnd), [digest_numpy(b.detach().numpy()) for b in self.buffers])
            return
        stream = torch.cuda.current_stream(self.device).cuda_stream
        for i, b in enumerate(self.buffers):
            rc = self.lib.gfk_digest_launch(
                C.c_void_p(b.data_ptr()), b.numel(), C.c_void_p(self._part.data_ptr()), self.nblk,
                C.c_void_p(self._out.data_ptr() + 8 * i), C.c_void_p(self._host.data_ptr() + 8 * i),
                C.c_void_p(stream))
            if rc:
                raise RuntimeError(f"gfk_digest_launch failed ({rc})")
        self._ev.record()
        self._pending = (int(rnd), None)

    def result(self) -> Optional[tuple]:
        p, self._pending = self._pending, None
        if p is None:
            return None
        if p[1] is not None:
            return p
        self._ev.synchronize()
        return p[0], [int(v) & (2 ** 64 - 1) for v in self._host.tolist()]


def compare(per_rank: List, rank: int) -> Optional[str]:
    """``per_rank``: every rank's ``(round, [digests])`` (all-gathered); None if all rounds
    match and every digest is equal, else a description of the divergence."""
    rounds = {r[0] for r in per_rank}
    if len(rounds) != 1:
        return f"ranks digested different rounds {sorted(rounds)}"
    ref = per_rank[0][1][0]
    bad = [(j, k) for j, (_, ds) in enumerate(per_rank) for k, d in enumerate(ds) if d != ref]
    if not bad:
        return None
    j, k = bad[0]
    return (f"shared state diverged across ranks after round {per_rank[0][0]}: rank {j} "
            f"client slot {k} digest {per_rank[j][1][k]:016x} vs rank 0 {ref:016x} "
            f"({len(bad)} differing buffer(s))")
