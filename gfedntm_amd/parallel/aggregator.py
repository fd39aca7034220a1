"""Sample-weighted FedAvg of the clients' shared state.

Reference semantics (src/federation/server.py:477-487): after every client did
one local step, each shared tensor becomes sum_i n_i W_i / sum_i n_i where
n_i is the client's document count; Adam moments stay local.

MI355X mapping: every client's shared state is one contiguous fp32 prefix of
its flat buffer (utils/flat.py).  The fused Adam kernel already multiplied it
by w_i = n_i / sum n (ops/engine.py ``set_fedavg_scale``), so the average is a
single in-place all-reduce(SUM) per round -- RCCL over xGMI on GPUs (backend
"nccl" is RCCL on ROCm), gloo on CPU.  Large states are split into buckets so
RCCL can pipeline them over its rings; ``async_op`` returns work handles so
the caller can overlap host bookkeeping with the collective.

``LocalAggregator`` is the in-process equivalent for N simulated clients
(tests, single-GPU simulations): it computes the exact weighted sum.
"""
from __future__ import annotations

import ctypes
import itertools
import time
from typing import List, Optional, Sequence

import numpy as np
import torch
import torch.distributed as dist


def fedavg_weights(n_samples: Sequence[int]) -> List[float]:
    tot = float(sum(n_samples))
    return [n / tot for n in n_samples]


class CollectiveAggregator:
    """All-reduce of pre-scaled flat buffers across the ranks of a process group.

    ``method``: "rccl" (torch.distributed all_reduce: RCCL on GPUs, gloo on CPU),
    "xgmi" (the custom two-shot peer-memory kernel, parallel/xgmi.py) or "auto":
    xgmi when the group is one node of <= 8 GPU ranks and the kernel passes its
    exactness check at :meth:`prepare`, RCCL otherwise.  The environment variable
    ``GFEDNTM_ALLREDUCE`` (rccl|xgmi|auto) overrides the default."""

    def __init__(self, group=None, bucket_bytes: int = 64 << 20, method: Optional[str] = None,
                 wire: str = "fp32", weight: Optional[float] = None):
        """``wire``: "fp32" (the reference's averaging: the sum of the pre-scaled states) or
        "bf16delta" (opt-in, half the bytes: bf16 departures of the rank's pre-scaled state
        from the last averaged state, ``weight`` = the rank's FedAvg weight sum; see
        csrc/comm.hip gfk_xgmi_allreduce_bf16d and :meth:`_delta_allreduce`)."""
        import os
        if wire not in ("fp32", "bf16delta"):
            raise ValueError("wire must be 'fp32' or 'bf16delta'")
        if wire == "bf16delta" and weight is None:
            raise ValueError("bf16delta needs this rank's FedAvg weight")
        self.wire = wire
        self.weight = None if weight is None else float(np.float32(weight))
        self.ref: Optional[torch.Tensor] = None      # bf16delta over RCCL / gloo
        self.group = group
        self.bucket_elems = max(1, bucket_bytes // 4)
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.method = (method or os.environ.get("GFEDNTM_ALLREDUCE", "auto")).lower()
        self.xgmi = None
        self.active = "rccl"
        self.tuning = None
        self.setup_s = 0.0
        self.fallback_reason = None      # why "auto" / "xgmi" did not get the xGMI kernel

    def prepare(self, flat: torch.Tensor, inplace: bool = False) -> str:
        """Choose the all-reduce for buffers shaped like ``flat`` (call once, on every
        rank, before the timed / captured region).  ``inplace``: the xGMI kernel maps
        ``flat`` itself into the peers (no stage copy; every later call must pass this
        very buffer).  Returns the method in use."""
        t_setup = time.perf_counter()
        if self.wire == "bf16delta":
            inplace = False                  # the peers read deltas, not the state
        initial = flat.detach().clone() if self.wire == "bf16delta" else None
        try:
            return self._prepare(flat, inplace)
        finally:
            self.setup_s = time.perf_counter() - t_setup
            if initial is not None:          # the last averaged state so far: the state itself
                self.set_reference(initial)

    def set_reference(self, t: torch.Tensor):
        """bf16delta: reset the last averaged state (W0 at setup; the loaded state after a
        checkpoint resume).  Identical on every rank."""
        if self.wire != "bf16delta":
            return
        if self.xgmi is not None:
            self.xgmi.set_reference(t)
        # (kept for the torch.distributed path as well: a call that falls through to it --
        # async, or another buffer size -- must start from the same reference on every rank)
        self.ref = t.detach().reshape(-1).clone()

    def _prepare(self, flat: torch.Tensor, inplace: bool = False) -> str:
        if self.world == 1 or self.method == "rccl" or flat.device.type != "cuda":
            self.active = "rccl"
            return self.active
        import socket
        hosts: List = [None] * self.world
        dist.all_gather_object(hosts, socket.gethostname(), group=self.group)
        ok = len(set(hosts)) == 1 and self.world <= 8
        xg = None
        if ok:
            from .xgmi import XgmiAllReduce
            try:
                xg = XgmiAllReduce(flat.numel(), flat.device, group=self.group,
                                   data=flat if inplace else None, wire=self.wire,
                                   weight=self.weight)
            except Exception as e:   # every rank must reach the agreement below
                import logging
                logging.getLogger("gfedntm_amd.xgmi").warning(
                    "xGMI all-reduce setup failed (RCCL instead): %s", e)
                self.fallback_reason = f"setup: {e}"
                xg = None
        flags: List = [None] * self.world
        dist.all_gather_object(flags, xg is not None, group=self.group)
        ok = ok and all(flags) and xg.validate()
        if ok and self.method == "auto" and dist.get_backend(self.group) == "nccl":
            # measured choice on this node: time both collectives on this size (the
            # slowest rank's time decides, so every rank takes the same branch).  The
            # xGMI kernel keeps a 10 % edge: it is captured in the step graph and
            # overlapped with the backward, RCCL runs after the step.
            # the warm-up launches run before the timing barrier, with the ranks only
            # loosely aligned: the generous validation spin bound, and a timed-out wait
            # (sticky error word) counts as a failed validation instead of surfacing as a
            # CommError after training
            spin = xg.c.spin_limit
            xg.c.spin_limit = max(spin, 1 << 26)
            saved = flat.clone() if inplace else None
            try:
                # (in-place: timed on the registered buffer itself, restored after)
                tx = self._time(xg.allreduce_, flat, on=flat if inplace else None)
            finally:
                xg.c.spin_limit = spin
                if saved is not None:
                    flat.copy_(saved)
                    del saved
            err = xg.error()
            tr = self._time((lambda b: dist.all_reduce(b, group=self.group)) if self.wire == "fp32"
                            else (lambda b: dist.all_reduce(b.to(torch.bfloat16), group=self.group)),
                            flat)
            t = torch.tensor([tx, tr, float(err != 0)], dtype=torch.float64, device=flat.device)
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
            tx, tr, bad = (float(v) for v in t.tolist())
            self.tuning = {"xgmi_ms": round(tx, 4), "rccl_ms": round(tr, 4),
                           "bytes": 4 * flat.numel()}
            if tr < 0.9 * tx or bad:
                ok = False
        if ok:
            self.xgmi, self.active = xg, "xgmi"
        else:
            if self.fallback_reason is None:
                self.fallback_reason = ("not one node of <= 8 ranks" if xg is None and self.world > 8
                                        else "measured slower than RCCL or failed validation")
            if xg is not None:
                xg.close()
            if self.method == "xgmi":
                raise RuntimeError("xGMI all-reduce requested but unavailable / failed validation")
            self.active = "rccl"
        return self.active

    def _time(self, fn, like: torch.Tensor, iters: int = 10, warmup: int = 3,
              on: Optional[torch.Tensor] = None) -> float:
        """Mean ms of ``fn`` (an in-place all-reduce) on a scratch buffer shaped like
        ``like`` (or on ``on``); every rank runs it the same number of times."""
        buf = torch.zeros_like(like) if on is None else on
        for _ in range(warmup):
            fn(buf)
        torch.cuda.synchronize(like.device)
        dist.barrier(group=self.group)
        t0 = time.perf_counter()
        for _ in range(iters):
            fn(buf)
        torch.cuda.synchronize(like.device)
        return (time.perf_counter() - t0) / iters * 1e3

    def describe(self) -> dict:
        """What the data plane of this buffer is (for the fedavg_attach records)."""
        d = {"method": self.active, "wire": self.wire}
        if self.xgmi is not None:
            d["inplace"] = self.xgmi.data is not None
            d["flags_uncached"] = self.xgmi.flags_uncached
            d["nblk"] = self.xgmi.nblk
        elif self.fallback_reason:
            d["fallback"] = self.fallback_reason
        return d

    def weights(self, n_local: int, device) -> List[float]:
        t = torch.tensor([float(n_local)], dtype=torch.float64, device=device)
        allv = [torch.zeros_like(t) for _ in range(self.world)]
        dist.all_gather(allv, t, group=self.group)
        return fedavg_weights([float(v.item()) for v in allv])

    def allreduce_(self, flat: torch.Tensor, async_op: bool = False):
        """In-place SUM of a (pre-scaled) flat buffer; returns work handles if async."""
        if self.world == 1:
            return []
        n = flat.numel()
        if self.xgmi is not None and n == self.xgmi.n and not async_op:
            self.xgmi.allreduce_(flat)
            return []
        if self.wire == "bf16delta":
            self._delta_allreduce(flat)
            return []
        works = []
        for a in range(0, n, self.bucket_elems):
            w = dist.all_reduce(flat[a: a + self.bucket_elems], op=dist.ReduceOp.SUM,
                                group=self.group, async_op=async_op)
            if async_op:
                works.append(w)
        return works

    def _delta_allreduce(self, flat: torch.Tensor):
        """bf16delta over torch.distributed (RCCL / gloo), with the xGMI kernel's arithmetic
        (csrc/comm.hip gfk_xgmi_allreduce_bf16d, LocalAggregator's golden): every rank's
        d_r = bf16(f_r - w_r ref) goes on the wire, the d_r are summed in fp32 IN RANK ORDER
        and the sum rounded once to bf16, S; W = ref + S, ref = W -- identical on every rank
        for any rank count.  (A native bf16 all-reduce would round after every add / ring
        hop, and its order depends on the ring.)  The d_r travel by all_gather as int32 pairs
        of bf16 words (bit-exact on every backend), one bucket at a time."""
        if self.ref is None:
            raise RuntimeError("bf16delta: no reference state (set_reference / prepare first)")
        ref = self.ref
        n = ref.numel()
        w = torch.tensor(self.weight, dtype=torch.float32, device=ref.device)
        out = flat.reshape(-1)
        step = max(2, self.bucket_elems - self.bucket_elems % 2)
        for a in range(0, n, step):
            b = min(n, a + step)
            d = (out[a:b] - ref[a:b] * w).to(torch.bfloat16)
            if d.numel() % 2:
                d = torch.cat([d, d.new_zeros(1)])
            words = d.view(torch.int32)
            got = [torch.empty_like(words) for _ in range(self.world)]
            dist.all_gather(got, words, group=self.group)
            s = got[0].view(torch.bfloat16).float()
            for g in got[1:]:
                s = s + g.view(torch.bfloat16).float()
            s = s.to(torch.bfloat16).float()[: b - a]
            out[a:b].copy_(ref[a:b] + s)
        ref.copy_(out)

    def average_(self, flat: torch.Tensor, weight: float):
        """Weighted average without a prior pre-scale (generic path)."""
        if self.world == 1:
            return
        flat.mul_(weight)
        self.allreduce_(flat)


class _GfkLocalAvg(ctypes.Structure):
    _fields_ = [("f", ctypes.c_void_p), ("gend", ctypes.c_void_p), ("off", ctypes.c_int64),
                ("n", ctypes.c_int64), ("n_clients", ctypes.c_int32), ("mode", ctypes.c_int32),
                ("n_groups", ctypes.c_int32), ("pad", ctypes.c_int32)]


LOCAL_ALL, LOCAL_FIRST, LOCAL_BCAST = 0, 1, 2     # gfk_local_fedavg modes (csrc/comm.hip)

# device tables of the in-process fold (client buffer pointers + group ends), one per
# (device, pointers, groups): built outside graph captures, kept alive for the graphs
# that baked their addresses in
_TABLES = {}


def _local_table(flats: Sequence[torch.Tensor], groups: Sequence[int]) -> torch.Tensor:
    dev = flats[0].device
    ptrs = tuple(int(f.data_ptr()) for f in flats)
    key = (str(dev), ptrs, tuple(groups))
    t = _TABLES.get(key)
    if t is None:
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError("local_fedavg: call prepare_local_fedavg() on these buffers "
                               "before the graph capture (its device table is uploaded once)")
        if any(p % 16 for p in ptrs):
            raise ValueError("local_fedavg buffers must be 16-byte aligned")
        ends = list(itertools.accumulate(int(g) for g in groups))
        # one int64 tensor: the pointers, then the group ends as int32 pairs
        host = torch.tensor([int(p) for p in ptrs], dtype=torch.int64)
        gend = torch.tensor(ends + [0] * (len(ends) & 1), dtype=torch.int32).view(torch.int64)
        t = torch.cat([host, gend]).to(dev)
        _TABLES[key] = t
    return t


def prepare_local_fedavg(flats: Sequence[torch.Tensor], groups: Optional[Sequence[int]] = None):
    """Upload the device table of ``flats`` (call before capturing local_fedavg)."""
    groups = [len(flats)] if groups is None else [int(g) for g in groups]
    return _local_table(flats, groups)


def local_fedavg(flats: Sequence[torch.Tensor], mode: int = LOCAL_ALL,
                 groups: Optional[Sequence[int]] = None, off: int = 0, n: Optional[int] = None):
    """One launch of csrc/comm.hip ``gfk_local_fedavg`` on the current stream (capture
    safe once :func:`prepare_local_fedavg` ran on the same buffers): the group-wise left-
    fold sum of ``flats`` (``groups``: sizes of consecutive client groups, default one
    group) written to every buffer (LOCAL_ALL) or to flats[0] only (LOCAL_FIRST), or
    flats[0] copied to the others (LOCAL_BCAST).  ``off`` / ``n``: the float range folded
    (default the whole buffers).  Any number of clients."""
    C = ctypes
    from ..ops import native
    lib = native.kernels()
    if not getattr(lib, "_gfk_local_avg_declared", False):
        lib.gfk_local_avg_struct_size.restype = C.c_size_t
        lib.gfk_local_fedavg_launch.argtypes = [C.POINTER(_GfkLocalAvg), C.c_int, C.c_void_p]
        if lib.gfk_local_avg_struct_size() != C.sizeof(_GfkLocalAvg):
            raise RuntimeError("GfkLocalAvg ABI mismatch between csrc/comm.hip and aggregator.py")
        lib._gfk_local_avg_declared = True
    groups = [len(flats)] if groups is None else [int(g) for g in groups]
    if sum(groups) != len(flats) or min(groups) < 1:
        raise ValueError(f"groups {groups} do not partition {len(flats)} clients")
    total = flats[0].numel()
    n = total - off if n is None else int(n)
    if off % 4 or off < 0 or off + n > total or any(f.numel() != total for f in flats):
        raise ValueError(f"bad local_fedavg range [{off}, {off + n}) of {total}")
    table = _local_table(flats, groups)
    d = _GfkLocalAvg()
    d.f = table.data_ptr()
    d.gend = table.data_ptr() + 8 * len(flats)
    d.off, d.n = int(off), n
    d.n_clients, d.mode, d.n_groups = len(flats), int(mode), len(groups)
    cu = torch.cuda.get_device_properties(flats[0].device).multi_processor_count
    grid = int(max(1, min(-(-n // 1024), 4 * cu)))
    stream = torch.cuda.current_stream(flats[0].device).cuda_stream
    rc = lib.gfk_local_fedavg_launch(C.byref(d), grid, C.c_void_p(stream))
    if rc:
        raise RuntimeError(f"gfk_local_fedavg_launch failed ({rc})")
    d._table = table
    return d


class LocalAggregator:
    """In-process FedAvg over N client flat buffers (exact reference order of ops).

    On a GPU, pre-scaled buffers of any number of clients are summed by one HIP kernel
    (csrc/comm.hip ``gfk_local_fedavg``: client-order sum written back to every
    client, capture-safe); the eager torch sequence is the CPU / oracle path.
    ``groups`` (sizes of consecutive client groups) sums group-wise first, then the
    group sums in order: the summation tree of the same clients spread over ranks
    (each rank folds its clients, the collective folds the ranks), so the in-process
    golden and the distributed run agree bit for bit."""

    def __init__(self, n_samples: Sequence[int], groups: Optional[Sequence[int]] = None,
                 wire: str = "fp32"):
        self.n = [int(x) for x in n_samples]
        self.w = fedavg_weights(self.n)
        self.groups = None if groups is None else [int(g) for g in groups]
        if self.groups is not None and sum(self.groups) != len(self.n):
            raise ValueError(f"groups {self.groups} do not partition {len(self.n)} clients")
        if wire not in ("fp32", "bf16delta"):
            raise ValueError("wire must be 'fp32' or 'bf16delta'")
        # bf16delta: the in-process golden of the distributed bf16-delta FedAvg -- every group
        # (default: every client) is one rank of csrc/comm.hip gfk_xgmi_allreduce_bf16d
        self.wire = wire
        self.ref: Optional[torch.Tensor] = None
        self._desc = None

    def set_reference(self, t: torch.Tensor):
        """bf16delta: the last averaged state (W0 at the start, or a resumed state)."""
        self.ref = t.detach().reshape(-1).clone()

    def group_weights(self) -> List[float]:
        """Every group's FedAvg weight sum as the float32 the ranks use."""
        groups = self.groups or [1] * len(self.n)
        out, j = [], 0
        for g in groups:
            out.append(float(np.float32(sum(self.w[j:j + g]))))
            j += g
        return out

    def _delta_(self, flats: Sequence[torch.Tensor]):
        """bf16delta round on pre-scaled client states: per group, d_g = bf16(fold_g - w_g ref);
        S = bf16(fp32 sum of the d_g in group order); every client <- ref + S = ref."""
        if self.ref is None:
            raise RuntimeError("bf16delta: set_reference(W0) first")
        ref = self.ref
        groups = self.groups or [1] * len(flats)
        s, j = None, 0
        for g, wg in zip(groups, self.group_weights()):
            part = flats[j].detach().reshape(-1).clone()
            for f in flats[j + 1:j + g]:
                part.add_(f.reshape(-1))
            j += g
            t = ref * torch.tensor(wg, dtype=torch.float32, device=ref.device)
            d = (part - t).to(torch.bfloat16).float()
            s = d if s is None else s + d
        ref.copy_(ref + s.to(torch.bfloat16).float())
        for f in flats:
            f.reshape(-1).copy_(ref)
        return flats[0]

    def _native(self, flats: Sequence[torch.Tensor]) -> bool:
        if flats[0].device.type != "cuda":
            return False
        n = flats[0].numel()
        return all(f.device == flats[0].device and f.dtype == torch.float32 and f.is_contiguous()
                   and f.numel() == n and f.data_ptr() % 16 == 0 for f in flats)

    def prepare(self, flats: Sequence[torch.Tensor]) -> bool:
        """Upload the fold's device table (before capturing :meth:`fused_sum_`)."""
        if len(flats) > 1 and self._native(flats):
            prepare_local_fedavg(flats, self.groups)
            return True
        return False

    def fused_sum_(self, flats: Sequence[torch.Tensor]):
        """flats[i] <- sum_j flats[j] (client order, group-wise) for all i, one kernel
        launch on the current stream.  Returns False when the buffers don't qualify
        (caller falls back)."""
        if self.wire != "fp32":
            return False
        if len(flats) == 1:
            return True
        if not self._native(flats):
            return False
        self._desc = local_fedavg(flats, LOCAL_ALL, self.groups)
        return True

    def average_(self, flats: Sequence[torch.Tensor], prescaled: bool = False,
                 out: Optional[torch.Tensor] = None):
        """flats[i] <- sum_j w_j flats[j] for all i (in place)."""
        if self.wire == "bf16delta":
            if not prescaled:
                for w, f in zip(self.w, flats):
                    f.mul_(w)
            return self._delta_(flats)
        if len(flats) == 1 and prescaled:
            return flats[0]
        if prescaled and out is None and self.fused_sum_(flats):
            return flats[0]
        acc = torch.zeros_like(flats[0]) if out is None else out.zero_()
        if self.groups is None:
            for w, f in zip(self.w, flats):
                if prescaled:
                    acc.add_(f)
                else:
                    acc.add_(f, alpha=w)
            for f in flats:
                f.copy_(acc)
            return acc
        groups = self.groups
        j = 0
        for gi, g in enumerate(groups):
            part = None
            for _ in range(g):
                f = flats[j] if prescaled else flats[j] * self.w[j]
                part = f.clone() if part is None else part.add_(f)
                j += 1
            if gi == 0:
                acc.copy_(part)
            else:
                acc.add_(part)
        for f in flats:
            f.copy_(acc)
        return acc
