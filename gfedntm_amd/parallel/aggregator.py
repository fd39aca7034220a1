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

from typing import List, Optional, Sequence

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

    def __init__(self, group=None, bucket_bytes: int = 64 << 20, method: Optional[str] = None):
        import os
        self.group = group
        self.bucket_elems = max(1, bucket_bytes // 4)
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.method = (method or os.environ.get("GFEDNTM_ALLREDUCE", "auto")).lower()
        self.xgmi = None
        self.active = "rccl"

    def prepare(self, flat: torch.Tensor) -> str:
        """Choose the all-reduce for buffers shaped like ``flat`` (call once, on every
        rank, before the timed / captured region).  Returns the method in use."""
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
                xg = XgmiAllReduce(flat.numel(), flat.device, group=self.group)
            except Exception as e:   # every rank must reach the agreement below
                import logging
                logging.getLogger("gfedntm_amd.xgmi").warning("xGMI all-reduce setup failed: %s", e)
                xg = None
        flags: List = [None] * self.world
        dist.all_gather_object(flags, xg is not None, group=self.group)
        ok = ok and all(flags) and xg.validate()
        if ok:
            self.xgmi, self.active = xg, "xgmi"
        else:
            if xg is not None:
                xg.close()
            if self.method == "xgmi":
                raise RuntimeError("xGMI all-reduce requested but unavailable / failed validation")
            self.active = "rccl"
        return self.active

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
        works = []
        for a in range(0, n, self.bucket_elems):
            w = dist.all_reduce(flat[a: a + self.bucket_elems], op=dist.ReduceOp.SUM,
                                group=self.group, async_op=async_op)
            if async_op:
                works.append(w)
        return works

    def average_(self, flat: torch.Tensor, weight: float):
        """Weighted average without a prior pre-scale (generic path)."""
        if self.world == 1:
            return
        flat.mul_(weight)
        self.allreduce_(flat)


class LocalAggregator:
    """In-process FedAvg over N client flat buffers (exact reference order of ops)."""

    def __init__(self, n_samples: Sequence[int]):
        self.n = [int(x) for x in n_samples]
        self.w = fedavg_weights(self.n)

    def average_(self, flats: Sequence[torch.Tensor], prescaled: bool = False,
                 out: Optional[torch.Tensor] = None):
        """flats[i] <- sum_j w_j flats[j] for all i (in place)."""
        acc = torch.zeros_like(flats[0]) if out is None else out.zero_()
        for w, f in zip(self.w, flats):
            if prescaled:
                acc.add_(f)
            else:
                acc.add_(f, alpha=w)
        for f in flats:
            f.copy_(acc)
        return acc
