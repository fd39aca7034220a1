"""More federated clients than ranks: hierarchical FedAvg.

The reference federates any number of clients (``--min_clients_federation``,
/root/reference/main.py:200,259; every round loops over all registered clients,
src/federation/server.py:442-484,500).  On one node the natural unit is one rank per
GPU, so with N clients on R < N ranks each rank hosts a contiguous block of clients:

  round r, rank q (clients i in block q):
    1. every local client does its local step -- fused engine: one launch per kernel
       phase for all local clients (ops/engine.py BatchedSteps, grid z = client), or one
       graph branch per client where the clients cannot be batched -- its shared state
       pre-scaled by its GLOBAL weight w_i = n_i / sum_all n;
    2. the rank folds its clients' states in client order into the first client's
       buffer (csrc/comm.hip gfk_local_fedavg, mode "first");
    3. the ranks all-reduce that partial sum (the xGMI two-shot kernel: rank-order
       fold; RCCL otherwise);
    4. the total is broadcast into the rank's other clients (mode "broadcast").

Steps 1-4 are one hipGraph per round when the collective is the xGMI kernel.  The sum
is fold_ranks(fold_clients_of_rank(w_i W_i)): the in-process golden with the same
grouping (``LocalFederation(..., groups=sizes)``, batched the same way) produces it bit
for bit.

Control plane (gloo): the ranks agree on the client-to-rank map (every rank announces
its client ids; they must partition 1..N in rank order), the vocabulary (union of every
client's terms) and the FedAvg weights (every client's document count).
"""
from __future__ import annotations

import datetime
import logging
import os
import time
from typing import Dict, List, Optional, Sequence

import torch

from ..data.vocab import union_vocabulary, vocabulary_dict
from ..eval.export import save_model_as_npz, server_model_path
from ..parallel.aggregator import (LOCAL_BCAST, LOCAL_FIRST, CollectiveAggregator,
                                   fedavg_weights, local_fedavg)
from ..utils import checkpoint as ckpt
from ..utils.config import DEFAULT_GRADS_TO_SHARE
from ..utils.logging import MetricsWriter
from ..utils.misc import graph_capture
from ..utils.trace import RoundWindow, trace_range
from .client import FederatedClient
from .data import ClientCorpus


def assign_clients(n_clients: int, world: int) -> List[List[int]]:
    """Client ids 1..n_clients in contiguous blocks over ``world`` ranks (the first
    n_clients % world ranks take one more)."""
    if world < 1 or n_clients < world:
        raise ValueError(f"{n_clients} clients cannot fill {world} ranks")
    base, extra = divmod(n_clients, world)
    out, c = [], 1
    for r in range(world):
        k = base + (1 if r < extra else 0)
        out.append(list(range(c, c + k)))
        c += k
    return out


def agree_client_map(local_ids: Sequence[int], world: int, group=None) -> List[List[int]]:
    """Every rank announces its client ids; they must be contiguous blocks that partition
    1..N in rank order (the summation tree the golden reproduces)."""
    import torch.distributed as dist
    allids: List = [None] * world
    dist.all_gather_object(allids, [int(i) for i in local_ids], group=group)
    flat = [i for ids in allids for i in ids]
    if flat != list(range(1, len(flat) + 1)) or any(len(ids) == 0 for ids in allids):
        raise RuntimeError(f"client-to-rank map {allids} is not a partition of 1..{len(flat)} "
                           "into non-empty contiguous blocks in rank order")
    return allids


class _RankRound:
    """One rank's round: local steps, in-rank fold, collective, broadcast."""

    def __init__(self, clients: List[FederatedClient], coll: Optional[CollectiveAggregator],
                 device, graph: bool):
        self.clients = clients
        self.coll = coll
        self.device = device
        self.shared = [c.shared for c in clients]
        engines = [c.tm.engine for c in clients]
        self.fused = all(c.fused for c in clients) and device.type == "cuda"
        self.coll_in_graph = coll is not None and coll.xgmi is not None
        self.graph = (graph and self.fused
                      and not any(e.host_gemm_fallback for e in engines))
        if self.graph:
            for c in clients:
                c.enable_graph(False)     # the round graph carries every client's step
        self._g = None
        self._gens = None
        self._streams = None

    def _fold_first(self):
        if len(self.shared) > 1:
            local_fedavg(self.shared, LOCAL_FIRST)

    def _bcast(self):
        if len(self.shared) > 1:
            local_fedavg(self.shared, LOCAL_BCAST)

    def _collective(self):
        if self.coll is not None:
            self.coll.allreduce_(self.shared[0])

    def _capture(self):
        engines = [c.tm.engine for c in self.clients]
        for e in engines:
            e.prepare_external_capture()
        g = torch.cuda.CUDAGraph()
        from ..ops.engine import BatchedSteps
        if os.environ.get("GFEDNTM_ROUND_BATCHED", "1") == "1" and BatchedSteps.possible(engines):
            # every local client's step in one launch per phase (grid z = client)
            bs = BatchedSteps(engines)
            bs.prepare()
            with graph_capture(g):
                bs.launch()
                self._fold_first()
                if self.coll_in_graph:
                    self._collective()
                    self._bcast()
            self._g, self._batched = g, bs
            self._gens = tuple(e.graph_gen for e in engines)
            return
        if self._streams is None:
            self._streams = [torch.cuda.Stream(self.device) for _ in engines]
        joins = [torch.cuda.Event() for _ in engines]
        with graph_capture(g):
            main = torch.cuda.current_stream(self.device)
            fork = torch.cuda.Event()
            fork.record(main)
            for e, st, ev in zip(engines, self._streams, joins):
                st.wait_event(fork)
                with torch.cuda.stream(st):
                    e.launch_step_phases()
                ev.record(st)
            for ev in joins:
                main.wait_event(ev)
            self._fold_first()
            if self.coll_in_graph:
                self._collective()
                self._bcast()
        self._g = g
        self._gens = tuple(e.graph_gen for e in engines)

    def step(self, it: int):
        if self.graph:
            engines = [c.tm.engine for c in self.clients]
            for e in engines:
                e.sync_step_counter(it)
            if self._g is not None and self._gens != tuple(e.graph_gen for e in engines):
                self._g = None
            if self._g is None:
                self._capture()
            self._g.replay()
            for e in engines:
                e.advance_host_step(it)
            if not self.coll_in_graph:
                self._collective()
                self._bcast()
            return
        for c in self.clients:
            c.local_step(it)
        if self.fused:
            self._fold_first()
            self._collective()
            self._bcast()
            return
        # CPU / torch engines: client-order fold, then the ranks' sum, then broadcast
        acc = self.shared[0]
        for f in self.shared[1:]:
            acc.add_(f)
        self._collective()
        for f in self.shared[1:]:
            f.copy_(acc)


def run_distributed_multi(corpora: Sequence[ClientCorpus], client_ids: Sequence[int], params: Dict,
                          model_type: str = "avitm", max_iters: int = 100, backend: str = "auto",
                          data_backend: Optional[str] = None,
                          grads_to_share: Sequence[str] = DEFAULT_GRADS_TO_SHARE, seed: int = 0,
                          save_client: Optional[str] = None, save_server: Optional[str] = None,
                          logger=None, graph: bool = True, log_every: int = 0,
                          stop_at_num_epochs: bool = False, checkpoint_dir: Optional[str] = None,
                          checkpoint_every: int = 0, stamp: Optional[str] = None,
                          metrics_path: Optional[str] = None, metrics_every: int = 0,
                          timing_warmup: int = 0, rehearse_1gpu: Optional[bool] = None,
                          allreduce: Optional[str] = None, round_hook=None) -> Dict:
    """This rank's block of clients in a federation of N clients over R ranks
    (torch.distributed initialised).  Same protocol, outputs and bookkeeping as
    :func:`~gfedntm_amd.federation.runner.run_distributed` (which it generalises to
    several clients per rank, parameter FedAvg only); rank 0 also saves the global
    model.  Returns the rank's clients."""
    import torch.distributed as dist
    from .runner import CTM_TYPES, CommError, build_dataset, make_topic_model, rehearsal_enabled
    if len(corpora) != len(client_ids) or not corpora:
        raise ValueError("one corpus per local client id")
    logger = logger or logging.getLogger("gfedntm_amd.federation")
    rank, world = dist.get_rank(), dist.get_world_size()
    data_backend = data_backend or dist.get_backend()
    rehearse = rehearsal_enabled() if rehearse_1gpu is None else bool(rehearse_1gpu)
    ctrl = dist.new_group(backend="gloo") if data_backend != "gloo" else None
    if data_backend == "nccl" or rehearse:
        device = torch.device("cuda", torch.cuda.current_device())
    else:
        device = torch.device("cpu")
    stamp = stamp or datetime.datetime.now().strftime("%Y%m%d")
    metrics = MetricsWriter(metrics_path)
    # ---- stage 1: client map, vocabulary union, weights (control plane) ----
    with trace_range("consensus"):
        cmap = agree_client_map(client_ids, world, group=ctrl)
        mine = [(c.local_terms(), c.n_docs) for c in corpora]
        gathered: List = [None] * world
        dist.all_gather_object(gathered, mine, group=ctrl)
    every = [x for g in gathered for x in g]              # client-id order
    terms = union_vocabulary([t for t, _ in every])
    vocab = vocabulary_dict(terms)
    weights = fedavg_weights([n for _, n in every])
    if rank == 0:
        logger.info("-- -- Global vocabulary agreed: %d terms from %d clients on %d ranks",
                    len(terms), len(every), world)
    clients: List[FederatedClient] = []
    for k, (cid, corpus) in enumerate(zip(client_ids, corpora)):
        ds = build_dataset(model_type, corpus, vocab, terms)
        tm = make_topic_model(model_type, params, len(terms), device, backend, grads_to_share,
                              seed=seed, logger=logger)
        if k == 0:
            with trace_range("w0_broadcast"):
                if data_backend == "gloo" and device.type == "cuda":
                    host = tm.flat.buffer.cpu()
                    dist.broadcast(host, src=0)
                    tm.flat.buffer.copy_(host)
                else:
                    dist.broadcast(tm.flat.buffer, src=0)
        else:
            tm.flat.buffer.copy_(clients[0].tm.flat.buffer)
        path = None
        if save_client is not None:
            from ..eval.export import client_model_path
            path = client_model_path(save_client, cid, stamp)
        c = FederatedClient(cid, tm, ds, max_iters, logger=logger, seed=seed + cid,
                            save_path=path, log_every=log_every,
                            epoch_snapshots=(model_type in CTM_TYPES))
        c.set_fedavg_weight(weights[cid - 1])
        c.enable_graph(graph)
        clients.append(c)
    # ---- data plane: the collective over the ranks' partial sums ----
    coll = None
    if world > 1:
        coll = CollectiveAggregator(method=allreduce if data_backend == "nccl" or rehearse
                                    else "rccl")
        coll.prepare(clients[0].shared)
        logger.info("-- -- FedAvg: %d local clients folded in-rank, %s across %d ranks",
                    len(clients), coll.active, world)
    rr = _RankRound(clients, coll, device, graph)
    start = 0
    if checkpoint_dir:
        starts = {ckpt.load_client_checkpoint(checkpoint_dir, c) for c in clients}
        if len(starts) != 1:
            raise RuntimeError(f"inconsistent client checkpoints on rank {rank}: {sorted(starts)}")
        start = starts.pop()
        rounds: List = [None] * world
        dist.all_gather_object(rounds, start, group=ctrl)
        if len(set(rounds)) != 1:
            raise RuntimeError(f"inconsistent client checkpoints: rounds {rounds}")
    # rounds where every rank meets (some client does long host work after them)
    plan_info: List = [None] * world
    dist.all_gather_object(plan_info, [(c.host_heavy_rounds(), c.done_round()) for c in clients],
                           group=ctrl)
    align, dones = set(), []
    for per_rank in plan_info:
        for heavy, d in per_rank:
            align.update(heavy)
            dones.append(d)
    stop_after = max_iters - 1
    if stop_at_num_epochs and all(d is not None for d in dones):
        stop_after = min(stop_after, max(dones))
    sync = (lambda: torch.cuda.synchronize(device)) if device.type == "cuda" else (lambda: None)

    def check_comm(where: str):
        err = coll.xgmi.error() if coll is not None and coll.xgmi is not None else 0
        flag = torch.tensor([int(err)], dtype=torch.int64)
        dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=ctrl)
        if int(flag.item()):
            raise CommError(f"rank {rank}: an xGMI all-reduce wait timed out before {where} "
                            f"(error {int(flag.item())}); the shared state is invalid")

    def meet(where: str):
        sync()
        check_comm(where)
        dist.barrier(group=ctrl)

    dist.barrier(group=ctrl)
    win = RoundWindow(sync)
    ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) \
        if (device.type == "cuda" and timing_warmup) else None
    t0 = time.perf_counter()
    timed_from, last = start, start - 1
    with trace_range("rounds"):
        for it in range(start, stop_after + 1):
            rr.step(it)
            heavy = it in align
            if heavy:
                sync()
                check_comm(f"the host work of round {it}")
            for c in clients:
                c.end_round(it)
            last = it
            if heavy:
                dist.barrier(group=ctrl)
            if round_hook is not None:
                round_hook(it)
            win.add(sum(int(c.plan.size[it]) for c in clients))
            if timing_warmup and it == start + timing_warmup - 1:
                meet("the timed region")
                t0 = time.perf_counter()
                if ev is not None:
                    ev[0].record()
                timed_from = it + 1
                win.reset()
            if metrics_every and (it + 1) % metrics_every == 0:
                w = win.close()
                check_comm(f"metrics window {it + 1}")
                metrics.write(event="window", rank=rank, round=it + 1, **w)
            if checkpoint_dir and checkpoint_every and (it + 1) % checkpoint_every == 0:
                with trace_range("checkpoint"):
                    meet(f"checkpoint {it + 1}")
                    for c in clients:
                        ckpt.save_client_checkpoint(checkpoint_dir, c, it + 1)
                    dist.barrier(group=ctrl)
    if ev is not None:
        ev[1].record()
    sync()
    wall = time.perf_counter() - t0
    device_s = ev[0].elapsed_time(ev[1]) * 1e-3 if ev is not None and timed_from > start else None
    check_comm("the end of training")
    n_rounds = last + 1 - timed_from
    docs = sum(int(c.plan.size[timed_from: last + 1].sum()) for c in clients) if n_rounds > 0 else 0
    for c in clients:
        c.flush()
    metrics.write(event="train_end", rank=rank, clients=list(client_ids), rounds=n_rounds,
                  wall_s=wall, docs=docs, docs_per_s=docs / wall if wall and docs else None,
                  ms_per_round=1e3 * wall / max(n_rounds, 1))
    for c in clients:
        if c.save_path and not c.results_saved:
            c.save_results(c.save_path)
    if rank == 0 and save_server:
        logger.info("-- -- Saving global model...")
        tm0 = clients[0].tm
        save_model_as_npz(server_model_path(save_server, stamp), tm0.get_topic_word_distribution(),
                          None, tm0.n_components, None)
    dist.barrier(group=ctrl)
    return {"rounds": last + 1, "timed_rounds": n_rounds, "wall_s": wall, "device_s": device_s,
            "docs": docs, "clients": clients, "client_map": cmap,
            "allreduce": None if coll is None else coll.active}
