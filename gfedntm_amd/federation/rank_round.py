"""One rank's round: its clients' local steps and the round's FedAvg.

The reference federates any number of clients (``--min_clients_federation``,
/root/reference/main.py:200,259); every round loops over all of them
(src/federation/server.py:442-484: pull every client's post-step state, :477-487:
the n_i-weighted average, :500-521: push it back).  On one node a rank drives one GPU,
so a rank hosts one client (N = R) or a contiguous block of them (N > R).  Both layouts
go through the same round loop (:func:`~gfedntm_amd.federation.runner.run_distributed`)
and one of the two classes below:

* :class:`SingleClientRound` -- the fused engine's own step with the FedAvg all-reduce
  inside it (graph-captured xGMI kernel, beta overlapped with the encoder backward) or
  right after it (RCCL / gloo), or classic gradient all-reduce (``agg_mode="grads"``);
* :class:`MultiClientRound` -- M clients' steps in ONE launch per kernel phase
  (ops/engine.py BatchedSteps, grid z = client), the in-rank fold of their pre-scaled
  states into the first client's buffer (csrc/comm.hip gfk_local_fedavg, any number of
  clients), the collective over the ranks' partial sums, the broadcast back -- one
  hipGraph per round with the xGMI kernel.  Beta's share is folded, all-reduced (in
  place for large states) and broadcast on a side stream as soon as the backward has
  finished it, overlapping the encoder backward and W_in update of all M clients, like
  the single-client step does.

The sum is fold_ranks(fold_clients_of_rank(w_i W_i)); ``LocalFederation(..., groups=
sizes)`` reproduces it bit for bit in one process.

Both expose the same failure-detection surface as the engine (error word of the xGMI
waits: synchronous, or copied asynchronously behind the enqueued rounds and polled), so
the runner's heartbeat, periodic polls and aligned checks work for either layout.
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional

import torch

from ..parallel.aggregator import (LOCAL_ALL, LOCAL_BCAST, LOCAL_FIRST, CollectiveAggregator,
                                   local_fedavg, prepare_local_fedavg)
from ..utils.misc import graph_capture
from .client import FederatedClient


def inplace_threshold_bytes() -> int:
    """Parts of at least this many bytes are all-reduced in place (xGMI maps the state
    itself into the peers instead of copying it into a stage first)."""
    return int(float(os.environ.get("GFEDNTM_XGMI_INPLACE_MB", "8")) * (1 << 20))


class SingleClientRound:
    """The rank's one client (N = R)."""

    def __init__(self, client: FederatedClient, world: int, device, on_gpu_plane: bool,
                 allreduce: Optional[str], agg_mode: str, bucket_bytes: int, logger,
                 wire: str = "fp32"):
        self.clients = [client]
        self.client = client
        self.agg_mode = agg_mode
        if wire != "fp32" and agg_mode != "params":
            raise ValueError("fedavg_wire bf16delta averages parameters (agg_mode 'params')")
        self.wire = wire
        self.agg = CollectiveAggregator(bucket_bytes=bucket_bytes, method="rccl", wire=wire,
                                        weight=client.weight if wire != "fp32" else None)
        self.agg.set_reference(client.shared)
        self.in_step = None
        if on_gpu_plane and client.fused and agg_mode == "params" and world > 1:
            self.in_step = client.tm.engine.attach_fedavg(method=allreduce, wire=wire)
            logger.info("-- -- FedAvg all-reduce: %s", self.in_step)
        self.method = self.in_step if self.in_step else (None if world == 1 else "rccl")
        self.attach = getattr(client.tm.engine, "fedavg_attach", None) if self.in_step else None

    @property
    def xgmi(self) -> bool:
        return bool(self.in_step) and self.in_step.startswith("xgmi")

    def rounds_per_replay(self) -> int:
        """Rounds one replay may carry (MultiClientRound.rounds_per_replay): the fused
        engine's k-step graph, the all-reduce inside it (or none: one rank)."""
        c = self.client
        if not (c.fused and self.agg_mode == "params" and c.tm.engine.steps_per_replay_ok()
                and (self.in_step is not None or self.agg.world == 1)):
            return 1
        return max(1, int(os.environ.get("GFEDNTM_ROUNDS_PER_GRAPH", "16")))

    def prewarm(self, kmax: int):
        """Capture the engine's 1, 2, 4, .. kmax-step graphs now (a capture inside the
        timed rounds costs milliseconds)."""
        e = self.client.tm.engine
        if self.rounds_per_replay() <= 1 or e.plan is None:
            return
        e.warm_graph()
        k = 2
        while k <= kmax:
            if k not in e._graphs_k:
                e._capture(k)
            k *= 2

    def step(self, it: int, hb=None, k: int = 1):
        """Enqueue round ``it`` (k > 1: rounds it .. it + k - 1 in one replay); ``hb``
        (parallel/heartbeat.py) is marked in the all-reduce phase once the local step is
        enqueued (a peer stuck before its step is then behind this rank)."""
        c = self.client
        if k > 1:
            if k > self.rounds_per_replay():
                raise ValueError(f"{k} rounds per replay on this round object")
            c.tm.engine.step_k(it, k)
            if hb is not None:
                for r in range(it, it + k):
                    hb.mark(r, 1)
            return
        c.local_step(it)
        if hb is not None:
            hb.mark(it, 1)
        if self.agg_mode == "grads":
            self.agg.allreduce_(c.shared_grads)
            c.apply_step(it)
            packed = c.pack_buffers()
            self.agg.allreduce_(packed)
            c.unpack_buffers(packed)
        elif self.in_step is None:
            self.agg.allreduce_(c.shared)

    def resync_reference(self):
        """bf16delta: the (loaded) shared state is the last averaged state."""
        if self.wire == "fp32":
            return
        self.agg.set_reference(self.client.shared)
        if self.in_step is not None:
            self.client.tm.engine.fedavg_set_reference()

    def error(self) -> int:
        e = self.client.tm.engine
        return e.fedavg_error() if self.in_step is not None and self.client.fused else 0

    def error_async(self):
        self.client.tm.engine.fedavg_error_async()

    def error_poll(self) -> int:
        return self.client.tm.engine.fedavg_error_poll()

    def debug(self) -> dict:
        return self.client.tm.engine.fedavg_debug() if self.in_step is not None else {}

    def close(self):
        if self.in_step is not None and self.client.fused:
            self.client.tm.engine.detach_fedavg()
            self.in_step = None


class MultiClientRound:
    """The rank's block of M > 1 clients (N > R)."""

    def __init__(self, clients: List[FederatedClient], world: int, device, on_gpu_plane: bool,
                 allreduce: Optional[str], graph: bool, logger, wire: str = "fp32"):
        self.clients = clients
        self.wire = wire
        # the rank's FedAvg weight: its clients' weights summed in client order (bf16delta)
        self.weight = sum(c.weight for c in clients) if wire != "fp32" else None
        self.device = device
        self.world = world
        self.shared = [c.shared for c in clients]
        engines = [c.tm.engine for c in clients]
        self.fused = all(c.fused for c in clients) and device.type == "cuda"
        n = self.shared[0].numel()
        # the shared state's parts: beta (final after the decoder backward in the fused
        # update mode), CombinedTM's adapt_bert (after ctx_bwd) and the rest, each with its
        # own collective (FusedEngine.fedavg_parts)
        self.parts: Dict[str, tuple] = {"rest": (0, n)}
        from ..ops.engine import UPDATE_FUSED
        if (self.fused and world > 1 and on_gpu_plane
                and all(e.update_mode == UPDATE_FUSED for e in engines)):
            self.parts = dict(engines[0].fedavg_parts())
        self.colls: Dict[str, CollectiveAggregator] = {}
        self.attach = None
        if world > 1:
            method = allreduce if on_gpu_plane else "rccl"
            big = inplace_threshold_bytes()
            for k, (a, b) in self.parts.items():
                coll = CollectiveAggregator(method=method, wire=wire, weight=self.weight)
                coll.prepare(self.shared[0][a:b], inplace=self.fused and 4 * (b - a) >= big)
                self.colls[k] = coll
            self.attach = {"s": round(sum(c.setup_s for c in self.colls.values()), 4),
                           "bytes": {k: 4 * (b - a) for k, (a, b) in self.parts.items()},
                           "inplace": {k: c.xgmi is not None and c.xgmi.data is not None
                                       for k, c in self.colls.items()},
                           "tuning": {k: c.tuning for k, c in self.colls.items() if c.tuning},
                           "plane": {k: c.describe() for k, c in self.colls.items()}}
        self.coll_in_graph = bool(self.colls) and all(c.xgmi is not None for c in self.colls.values())
        if not self.coll_in_graph and len(self.parts) > 1:
            # one RCCL all-reduce of the whole state after the round graph
            for c in self.colls.values():
                if c.xgmi is not None:
                    c.xgmi.close()
                    c.xgmi = None
            self.parts = {"rest": (0, n)}
            coll = CollectiveAggregator(method="rccl", wire=wire, weight=self.weight)
            coll.prepare(self.shared[0])
            self.colls = {"rest": coll}
        self.method = (None if world == 1 else
                       "xgmi" + ("+overlap" if len(self.parts) > 1 else "")
                       if self.coll_in_graph else self.colls["rest"].active)
        self.graph = (graph and self.fused and not any(e.host_gemm_fallback for e in engines))
        if self.graph:
            for c in clients:
                c.enable_graph(False)     # the round graph carries every client's step
        if self.fused:
            prepare_local_fedavg(self.shared)
        self.fold_plan: Optional[str] = None   # the in-rank FedAvg of the batched round
        self._g = None                    # the one-round graph
        self._gk: Dict[int, object] = {}  # k-round graphs (k > 1)
        self._bss: Dict[int, object] = {}  # the BatchedSteps each graph was captured with
        self._gens = None
        self._streams = None
        self._side = None
        self._err = None
        if logger is not None:
            logger.info("-- -- FedAvg: %d local clients folded in-rank, %s across %d ranks",
                        len(clients), self.method or "no collective", world)

    def _states_equal(self) -> bool:
        """Every client's shared state is the same (the in-epilogue fold reads client 0's
        copy for all of them): true after W0's broadcast and after every FedAvg."""
        s0 = self.shared[0]
        return all(torch.equal(s0, s) for s in self.shared[1:])

    # ---- pieces of the round (enqueued on the current stream) ----
    def _fold(self, part: str, mode: int):
        a, b = self.parts[part]
        if len(self.shared) > 1 and b > a:
            local_fedavg(self.shared, mode, off=a, n=b - a)

    def _reduce_part(self, part: str):
        """Fold the rank's clients, sum over the ranks, broadcast back (one part)."""
        if not self.colls:
            self._fold(part, LOCAL_ALL)
            return
        self._fold(part, LOCAL_FIRST)
        a, b = self.parts[part]
        self.colls[part].allreduce_(self.shared[0][a:b])
        self._fold(part, LOCAL_BCAST)

    def _fork(self, part: str):
        """``part``'s fold + all-reduce + broadcast on the side stream, from this point of
        the main stream (the side stream runs the forked parts in order)."""
        main = torch.cuda.current_stream(self.device)
        side, ev_join, forks = self._side
        ev = forks[part]
        ev.record(main)
        side.wait_event(ev)
        with torch.cuda.stream(side):
            self._reduce_part(part)
        ev_join.record(side)

    def rounds_per_replay(self) -> int:
        """Rounds one graph replay may carry (GFEDNTM_ROUNDS_PER_GRAPH, default 16): every
        round is device-driven (the batch, the step counter, the FedAvg and the in-graph
        xGMI all-reduce), so k consecutive rounds captured back to back are the same work
        as k replays of the one-round graph -- without the k - 1 graph-to-graph dispatch
        gaps (~8 us each between one-round replays at 8 clients, 0.125 ms rounds).  1 when
        something runs between rounds (RCCL outside the graph, the eager path)."""
        if not self.graph or (self.colls and not self.coll_in_graph):
            return 1
        return max(1, int(os.environ.get("GFEDNTM_ROUNDS_PER_GRAPH", "16")))

    def prewarm(self, kmax: int):
        """Capture the 1, 2, 4, .. kmax-round graphs now (SingleClientRound.prewarm)."""
        if self.rounds_per_replay() <= 1:
            return
        engines = [c.tm.engine for c in self.clients]
        if self._gens != tuple(e.graph_gen for e in engines):
            self._g = None
            self._gk.clear()
            self._bss.clear()
        if self._g is None:
            self._capture()
        k = 2
        while k <= kmax:
            if k not in self._gk:
                self._capture(k)
            k *= 2

    def _capture(self, k: int = 1):
        engines = [c.tm.engine for c in self.clients]
        for e in engines:
            e.prepare_external_capture()
        g = torch.cuda.CUDAGraph()
        from ..ops.engine import BatchedSteps
        batched = (os.environ.get("GFEDNTM_ROUND_BATCHED", "1") == "1"
                   and BatchedSteps.possible(engines))
        if self._side is None:
            self._side = (torch.cuda.Stream(self.device), torch.cuda.Event(),
                          {k: torch.cuda.Event() for k in ("beta", "wa")})
        if batched:
            bs = BatchedSteps(engines)
            bs.prepare()
            # one rank, GFEDNTM_FOLD=1: the round's FedAvg inside the update kernels' epilogues
            # (every client starts each round from the same averaged state) -- bit-identical
            # to the default, the batched steps + the fold kernel, but measured slower at the
            # headline (0.1355 vs 0.1174 ms per round, profiles/r6/README.md): opt-in
            fold = None
            self.fold_plan = "fold kernel" + (" + all-reduce" if self.colls else "")
            if not self.colls and os.environ.get("GFEDNTM_FOLD", "0") == "1":
                why = bs.fold_reason()
                if why is None and self._states_equal():
                    from ..ops import kernel_abi as abi
                    bs.set_fold(abi.FOLD_ALL)
                    fold = "in-epilogue"
                    self.fold_plan = fold
                else:
                    self.fold_plan = "fold kernel (%s)" % (why or "client states differ")
            # beta's / adapt_bert's shares on the side stream once the backward has
            # finished them (else reduced with the rest at the end of the round: the same
            # arithmetic)
            hooks, forked = {}, set()
            if self.coll_in_graph:
                for part, at in (("beta", bs.beta_final_phase()), ("wa", bs.wa_final_phase())):
                    if part in self.parts and at is not None:
                        hooks[at] = (lambda p=part: self._fork(p))
                        forked.add(part)
            with graph_capture(g):
                for _ in range(k):
                    bs.launch(after=hooks or None)
                    if fold is not None:
                        continue              # the FedAvg ran in the update epilogues
                    if self.coll_in_graph or not self.colls:
                        for part in self.parts:
                            if part not in forked:
                                self._reduce_part(part)
                        if forked:
                            torch.cuda.current_stream(self.device).wait_event(self._side[1])
                    else:
                        self._fold("rest", LOCAL_FIRST)
            self._batched = bs
            self._bss[k] = bs             # (its device tables are baked into the graph)
        else:
            self.fold_plan = "per-client graph branches + fold kernel"
            if self._streams is None:
                self._streams = [torch.cuda.Stream(self.device) for _ in engines]
            joins = [torch.cuda.Event() for _ in engines]
            with graph_capture(g):
                main = torch.cuda.current_stream(self.device)
                fork = torch.cuda.Event()
                for _ in range(k):
                    fork.record(main)
                    for e, st, ev in zip(engines, self._streams, joins):
                        st.wait_event(fork)
                        with torch.cuda.stream(st):
                            e.launch_step_phases()
                        ev.record(st)
                    for ev in joins:
                        main.wait_event(ev)
                    if self.coll_in_graph or not self.colls:
                        for part in self.parts:
                            self._reduce_part(part)
                    else:
                        self._fold("rest", LOCAL_FIRST)
        if k == 1:
            self._g = g
        else:
            self._gk[k] = g
        self._gens = tuple(e.graph_gen for e in engines)

    def step(self, it: int, hb=None, k: int = 1):
        """Rounds it .. it + k - 1 (k > 1: one replay of the k-round graph; the caller
        keeps every round that needs the host between rounds out of such a run)."""
        if k > 1:
            if not self.graph or k > self.rounds_per_replay():
                raise ValueError(f"{k} rounds per replay on this round object")
            engines = [c.tm.engine for c in self.clients]
            for e in engines:
                e.sync_step_counter(it)
            if self._gens != tuple(e.graph_gen for e in engines):
                self._g = None
                self._gk.clear()
                self._bss.clear()
            if k not in self._gk:
                self._capture(k)
            self._gk[k].replay()
            for e in engines:
                e.advance_host_step(it + k - 1)
            if hb is not None:
                for r in range(it, it + k):
                    hb.mark(r, 1)
            return
        self._step1(it, hb)

    def _step1(self, it: int, hb=None):
        if self.graph:
            engines = [c.tm.engine for c in self.clients]
            for e in engines:
                e.sync_step_counter(it)
            if self._gens != tuple(e.graph_gen for e in engines):
                self._g = None
                self._gk.clear()
                self._bss.clear()
            if self._g is None:
                self._capture()
            self._g.replay()
            for e in engines:
                e.advance_host_step(it)
            if hb is not None:
                hb.mark(it, 1)
            if self.colls and not self.coll_in_graph:
                # RCCL after the replay (the graph left the rank's partial sum in client 1)
                self.colls["rest"].allreduce_(self.shared[0])
                self._fold("rest", LOCAL_BCAST)
            return
        for c in self.clients:
            c.local_step(it)
        if hb is not None:
            hb.mark(it, 1)
        if self.fused:
            for part in self.parts:
                self._reduce_part(part)
            return
        # CPU / torch engines: client-order fold, then the ranks' sum, then broadcast
        acc = self.shared[0]
        for f in self.shared[1:]:
            acc.add_(f)
        if self.colls:
            self.colls["rest"].allreduce_(acc)
        for f in self.shared[1:]:
            f.copy_(acc)

    def time_local_steps(self, s0: int, n: int) -> Optional[float]:
        """Device milliseconds of the rank's batched local steps ALONE -- every client's step
        kernels with per-client updates, no FedAvg (neither the in-rank fold nor the
        collective) -- per round, replaying steps s0 .. s0 + n - 1 of the plan: the compute
        part of bench.py's round split.  The clients' states diverge: call after the run."""
        if not (self.fused and self.graph):
            return None
        from ..ops.engine import BatchedSteps
        engines = [c.tm.engine for c in self.clients]
        if not BatchedSteps.possible(engines):
            return None
        for e in engines:
            e.prepare_external_capture()
        bs = BatchedSteps(engines)
        bs.prepare()
        g = torch.cuda.CUDAGraph()
        with graph_capture(g):
            bs.launch()
        for e in engines:
            e.sync_step_counter(s0)
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize(self.device)
        ev0.record()
        for _ in range(n):
            g.replay()
        ev1.record()
        torch.cuda.synchronize(self.device)
        for e in engines:
            e.advance_host_step(s0 + n - 1)
        return ev0.elapsed_time(ev1) / max(n, 1)

    def resync_reference(self):
        """bf16delta: the (loaded) shared state is the last averaged state."""
        for k, coll in self.colls.items():
            a, b = self.parts[k]
            coll.set_reference(self.shared[0][a:b])

    # ---- failure detection (the engine's surface, over this rank's collectives) ----
    def _xgmis(self):
        return [c.xgmi for c in self.colls.values() if c.xgmi is not None]

    @property
    def xgmi(self) -> bool:
        return bool(self._xgmis())

    def error(self) -> int:
        err = 0
        for x in self._xgmis():
            err = err or x.error()
        return err

    def error_async(self):
        xs = self._xgmis()
        if not xs:
            return
        if self._err is None:
            self._err = {"host": torch.zeros(len(xs), dtype=torch.int32, pin_memory=True),
                         "ev": torch.cuda.Event(), "pending": False}
        for i, x in enumerate(xs):
            x.error_async(self._err["host"][i:i + 1])
        self._err["ev"].record()
        self._err["pending"] = True

    def error_poll(self) -> int:
        e = self._err
        if not e or not e["pending"] or not e["ev"].query():
            return 0
        e["pending"] = False
        return int(e["host"].max().item())

    def debug(self) -> dict:
        return {k: c.xgmi.debug_state() for k, c in self.colls.items() if c.xgmi is not None}

    def close(self):
        self._g = None
        self._gk.clear()
        self._bss.clear()
        for c in self.colls.values():
            if c.xgmi is not None:
                c.xgmi.close()
                c.xgmi = None
