"""Federated training runners.

The protocol (reference src/federation/{server,client}.py):

  stage 1  every client computes its local vocabulary; the global vocabulary is
           the sorted union; every client re-vectorises its corpus with it; the
           clients' document counts n_i give the FedAvg weights w_i = n_i / sum n;
           one initial model W0 (and fresh Adam state) is shared by everybody;
  stage 2  ``max_iters`` rounds: every client does one local minibatch step, the
           shared state (``grads_to_share`` intersected with the state_dict: all
           parameters and batch-norm buffers by default) becomes sum_i w_i W_i
           on every client; Adam moments stay local;
  stop     every client saves its results (npz), the coordinator saves the
           global model.

Transports:
  * :class:`LocalFederation` -- all clients in one process (CPU tests, single-GPU
    simulation of N clients), exact in-process weighted sum;
  * :func:`run_distributed` -- one process per client (torch.distributed):
    RCCL over xGMI for the data plane (backend "nccl" is RCCL on ROCm) or gloo on
    CPU, a gloo group for the control plane (vocabulary objects, counts);
  * the gRPC transport speaking the reference wire protocol lives in
    :mod:`gfedntm_amd.federation.grpc_transport`.

Reference defects fixed here: B1 (server model construction), B2 (shared keys are
intersected with the state_dict), B4/B5 (the global model is the averaged state,
saved at the end), B13 (no sleeps), B16 (results are saved once; optional stop).
"""
from __future__ import annotations

import datetime
import logging
import os
import time
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from ..data.bow import BOWDataset, CTMDataset
from ..data.vocab import union_vocabulary, vocabulary_dict
from ..eval.export import save_model_as_npz, server_model_path
from ..parallel.aggregator import CollectiveAggregator, LocalAggregator, fedavg_weights
from ..utils import checkpoint as ckpt
from ..utils.config import DEFAULT_GRADS_TO_SHARE, model_kwargs_from_params
from ..utils.logging import MetricsWriter
from ..utils.misc import graph_capture
from ..utils.trace import RoundWindow, trace_range
from .client import FederatedClient
from .data import ClientCorpus


CTM_TYPES = ("ctm", "zeroshot")


def shared_keys_for(model, grads_to_share: Sequence[str]) -> List[str]:
    """grads_to_share intersected with the state_dict (B2), in state_dict order."""
    want = set(grads_to_share)
    return [k for k in model.state_dict().keys() if k in want]


def make_topic_model(model_type: str, params: Dict, input_size: int, device,
                     backend: str = "auto", grads_to_share: Sequence[str] = DEFAULT_GRADS_TO_SHARE,
                     contextual_size: Optional[int] = None, seed: Optional[int] = None,
                     logger=None):
    """AVITM (``model_type='avitm'``, ProdLDA / NeuralLDA per params['model_type'])
    or CTM (``'ctm'``: CombinedTM, the reference's only federated CTM variant;
    ``'zeroshot'``: ZeroShotTM, same protocol)."""
    from ..models import AVITM, CombinedTM, ZeroShotTM
    kw = model_kwargs_from_params(params)
    kw.setdefault("model_type", "prodLDA")
    kw["verbose"] = False
    if model_type == "avitm":
        cls = AVITM
    elif model_type in CTM_TYPES:
        cls = CombinedTM if model_type == "ctm" else ZeroShotTM
        kw["contextual_size"] = int(contextual_size or params.get("contextual_size", 768))
    else:
        raise ValueError("model_type must be 'avitm', 'ctm' or 'zeroshot'")
    if seed is not None:
        torch.manual_seed(seed)
    # FlatState intersects grads_to_share with the state_dict (B2)
    return cls(input_size=input_size, backend=backend, device=device,
               shared_keys=list(grads_to_share) if grads_to_share is not None else None,
               seed=seed, logger=logger, **kw)


def build_dataset(model_type: str, corpus: ClientCorpus, vocab: Dict[str, int], terms: List[str]):
    X = corpus.bow(vocab)
    idx2token = {i: t for i, t in enumerate(terms)}
    if model_type in CTM_TYPES:
        if corpus.embeddings is None:
            raise ValueError("CTM needs contextual embeddings in the client corpus")
        return CTMDataset(corpus.embeddings, X, idx2token)
    return BOWDataset(X, idx2token)


def term_window(clients, it: int, w: Dict) -> Dict:
    """Mean loss / KL / RL of the window's rounds (ending at round ``it``), averaged over
    ``clients`` (reference federated_avitm.py:109 logs the minibatch loss)."""
    n = max(1, int(w.get("rounds") or 1))
    vals = [c.tm.engine.term_means(max(0, it + 1 - n), it + 1) for c in clients]
    out = {}
    for i, k in enumerate(("loss", "kl", "rl")):
        xs = [v[i] for v in vals if v[i] is not None]
        if xs:
            out[k] = float(np.mean(xs))
    return out


def record_terms(clients, on: bool):
    """KL / RL histories next to the loss (before any graph capture)."""
    if on:
        for c in clients:
            c.tm.engine.record_terms(True)


class LocalFederation:
    """N clients in one process; the shared state is averaged exactly after every round."""

    def __init__(self, corpora: Sequence[ClientCorpus], params: Dict, model_type: str = "avitm",
                 max_iters: int = 100, device=None, backend: str = "auto",
                 grads_to_share: Sequence[str] = DEFAULT_GRADS_TO_SHARE, seed: int = 0,
                 save_client: Optional[str] = None, save_server: Optional[str] = None,
                 logger=None, graph: bool = True, log_every: int = 0,
                 stop_at_num_epochs: bool = False, checkpoint_dir: Optional[str] = None,
                 checkpoint_every: int = 0, stamp: Optional[str] = None,
                 metrics_path: Optional[str] = None, metrics_every: int = 0, agg: str = "params",
                 round_graph: Optional[bool] = None, round_streams: bool = True,
                 groups: Optional[Sequence[int]] = None, round_batched: Optional[bool] = None,
                 fedavg_wire: str = "fp32"):
        self.logger = logger or logging.getLogger("gfedntm_amd.federation")
        self.agg_mode = agg
        if fedavg_wire != "fp32" and agg != "params":
            raise ValueError("fedavg_wire bf16delta averages parameters (agg 'params')")
        self.metrics = MetricsWriter(metrics_path)
        self.metrics_every = int(metrics_every)
        self.device = torch.device(device) if device is not None else \
            torch.device("cuda" if torch.cuda.is_available() else "cpu")
        self.max_iters, self.model_type = max_iters, model_type
        self.save_server, self.stop_at_num_epochs = save_server, stop_at_num_epochs
        self.checkpoint_dir, self.checkpoint_every = checkpoint_dir, checkpoint_every
        self.stamp = stamp or datetime.datetime.now().strftime("%Y%m%d")
        # ---- stage 1: vocabulary consensus ----
        with trace_range("consensus"):
            self.terms = union_vocabulary([c.local_terms() for c in corpora])
        self.vocab = vocabulary_dict(self.terms)
        self.logger.info("-- -- Global vocabulary agreed: %d terms from %d clients",
                         len(self.terms), len(corpora))
        datasets = [build_dataset(model_type, c, self.vocab, self.terms) for c in corpora]
        n = [len(d) for d in datasets]
        self.weights = fedavg_weights(n)
        # ---- identical W0 on every client ----
        self.clients: List[FederatedClient] = []
        for i, ds in enumerate(datasets):
            tm = make_topic_model(model_type, params, len(self.terms), self.device, backend,
                                  grads_to_share, seed=seed, logger=self.logger)
            if self.clients:     # the flat buffer holds every float parameter and buffer
                tm.flat.buffer.copy_(self.clients[0].tm.flat.buffer)
            cid = i + 1
            path = None
            if save_client is not None:
                from ..eval.export import client_model_path
                path = client_model_path(save_client, cid, self.stamp)
            c = FederatedClient(cid, tm, ds, max_iters, logger=self.logger, seed=seed + cid,
                                save_path=path, log_every=log_every,
                                epoch_snapshots=(model_type in CTM_TYPES), agg=agg)
            c.set_fedavg_weight(self.weights[i])
            c.ground_truth = corpora[i].ground_truth()
            c.enable_graph(graph and agg == "params")
            self.clients.append(c)
        # groups: client-block sizes of a multi-rank layout (hierarchical/run_distributed_multi)
        # -- the FedAvg sums each block first, then the block sums, in that run's order
        # fedavg_wire "bf16delta": the in-process golden of the reduced-byte FedAvg (every
        # group -- by default every client -- one rank); eager rounds
        record_terms(self.clients, bool(self.metrics_every or log_every))
        self.agg = LocalAggregator(n, groups, wire=fedavg_wire)
        self.agg.set_reference(self.clients[0].shared)
        # fused clients on one GPU: every client's step and the FedAvg kernel are
        # captured into ONE hipGraph per round (one replay instead of N step graphs
        # plus the eager aggregation), each client on its own stream: parallel graph
        # branches joined before the FedAvg kernel (8 clients: 0.35 ms / round
        # with branches vs 0.49 ms serialised, profiles/sim_clients.md)
        # (engines on the CTM host-GEMM fallback stay out of it: their hipBLASLt GEMMs
        # would run for the first time on the capture's per-client branch streams)
        can = (agg == "params" and graph and self.device.type == "cuda" and fedavg_wire == "fp32"
               and all(c.fused and not c.tm.engine.host_gemm_fallback for c in self.clients)
               and len(self.clients) > 1
               and self.agg._native([c.shared for c in self.clients]))
        self.round_graph = can if round_graph is None else (bool(round_graph) and can)
        self.round_streams = bool(round_streams)
        # batched kernels (one launch per phase for every client, csrc grid z = client);
        # GFEDNTM_ROUND_BATCHED=0 keeps one graph branch per client
        self.round_batched = (round_batched if round_batched is not None else
                              os.environ.get("GFEDNTM_ROUND_BATCHED", "1") == "1")
        self._batched = None
        self.fold_plan: Optional[str] = None    # the batched round's FedAvg (in-epilogue / kernel)
        self._rg = None
        self._rgk = {}                    # k -> (the k-round graph, the launches it baked in)
        self._rg_gens = None
        self._stop = False
        if self.round_graph:
            for c in self.clients:
                c.enable_graph(False)
        self.round = 0
        if checkpoint_dir:
            starts = {ckpt.load_client_checkpoint(checkpoint_dir, c) for c in self.clients}
            if len(starts) != 1:
                raise RuntimeError(f"inconsistent client checkpoints: rounds {sorted(starts)}")
            self.round = starts.pop()
            if self.round:
                self.logger.info("-- -- Resuming the federation at round %d", self.round)
            self.agg.set_reference(self.clients[0].shared)

    def _sync(self):
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)

    def _capture_round(self, k: int = 1):
        engines = [c.tm.engine for c in self.clients]
        for e in engines:
            e.prepare_external_capture()
        g = torch.cuda.CUDAGraph()
        shared = [c.shared for c in self.clients]
        self.agg.prepare(shared)          # the FedAvg kernel's device table, before capturing
        self._batched = None
        if self.round_batched:
            from ..ops.engine import BatchedSteps
            # groups (the golden of a multi-rank layout): one batched launch per group, as
            # each rank batches its own clients -- the launch plan (grid fill, backward
            # slabs) depends on the client count and fixes the summation order, so the
            # golden mirrors it to stay bit-identical to the ranks
            sizes = self.agg.groups or [len(engines)]
            parts, o = [], 0
            for s in sizes:
                parts.append(engines[o:o + s])
                o += s
            if all(BatchedSteps.possible(p) for p in parts):
                # one launch per phase for all clients (grid z = client), then the FedAvg kernel
                self._batched_parts = [BatchedSteps(p) for p in parts]
                self._batched = self._batched_parts[0]
                for b in self._batched_parts:
                    b.prepare()
                # one group, GFEDNTM_FOLD=1: the FedAvg inside the update kernels' epilogues
                # (rank_round.MultiClientRound: opt-in, measured slower than the fold kernel)
                fold = (len(self._batched_parts) == 1 and os.environ.get("GFEDNTM_FOLD", "0") == "1"
                        and self._batched.fold_reason() is None
                        and all(torch.equal(shared[0], x) for x in shared[1:]))
                if fold:
                    from ..ops import kernel_abi as abi
                    self._batched.set_fold(abi.FOLD_ALL)
                self.fold_plan = "in-epilogue" if fold else "fold kernel"
                with graph_capture(g):
                    for _ in range(k):
                        for b in self._batched_parts:
                            b.launch()
                        if not fold and not self.agg.fused_sum_(shared):
                            raise RuntimeError("round graph needs the native FedAvg kernel")
                self._store_round_graph(g, k)
                return
        if self.round_streams:
            streams = [torch.cuda.Stream(self.device) for _ in engines]
            joins = [torch.cuda.Event() for _ in engines]
        with graph_capture(g):
            main = torch.cuda.current_stream(self.device)
            fork = torch.cuda.Event()
            for _ in range(k):
                if self.round_streams:
                    fork.record(main)
                    for e, st, ev in zip(engines, streams, joins):
                        st.wait_event(fork)
                        with torch.cuda.stream(st):
                            e.launch_step_phases()
                        ev.record(st)
                    for ev in joins:
                        main.wait_event(ev)
                else:
                    for e in engines:
                        e.launch_step_phases()
                if not self.agg.fused_sum_(shared):
                    raise RuntimeError("round graph needs the native FedAvg kernel")
        self._store_round_graph(g, k)

    def _store_round_graph(self, g, k: int):
        if self._rg_gens != self._engine_gens():
            self._rgk = {}
        self._rgk[k] = (g, self._batched_parts if self._batched is not None else None)
        if k == 1:
            self._rg = g
        self._rg_gens = self._engine_gens()

    def _engine_gens(self):
        return tuple(c.tm.engine.graph_gen for c in self.clients)

    def _round_graph_step(self, it: int, k: int = 1):
        for c in self.clients:
            c.tm.engine.sync_step_counter(it)     # no-op unless resuming / out of sequence
        if self._rg_gens != self._engine_gens():
            self._rg, self._rgk = None, {}  # an engine was rebound / reconfigured since the capture
        if k not in self._rgk:
            self._capture_round(k)
        self._rgk[k][0].replay()
        for c in self.clients:
            c.tm.engine.advance_host_step(it + k - 1)

    def prewarm(self, kmax: int):
        """Capture the 1, 2, 4, .. kmax-round graphs now: a capture costs milliseconds,
        which must not land inside timed rounds."""
        if self._rg_gens != self._engine_gens():
            self._rg, self._rgk = None, {}
        k = 1
        while k <= kmax:
            if k not in self._rgk:
                self._capture_round(k)
            k *= 2

    def rounds_per_replay(self) -> int:
        """Rounds one replay of the round graph may carry (rank_round.MultiClientRound.
        rounds_per_replay; GFEDNTM_ROUNDS_PER_GRAPH, default 16)."""
        if not self.round_graph:
            return 1
        return max(1, int(os.environ.get("GFEDNTM_ROUNDS_PER_GRAPH", "16")))

    def _run_end(self, it: int, kmax: int, ends, timed_end: int) -> int:
        r = it
        while r < it + kmax - 1 and r not in ends and r != timed_end:
            n1 = r + 1
            if ((self.metrics_every and n1 % self.metrics_every == 0)
                    or (self.checkpoint_dir and self.checkpoint_every
                        and n1 % self.checkpoint_every == 0)):
                break
            r += 1
        return r

    def _round(self, it: int, k: int = 1):
        """Every client's local step and the FedAvg of round ``it`` (enqueued; k > 1:
        rounds it .. it + k - 1 in one replay of the round graph)."""
        if self.round_graph:
            self._round_graph_step(it, k)
            return
        for c in self.clients:
            c.local_step(it)
        if self.agg_mode == "grads":
            self.agg.average_([c.shared_grads for c in self.clients], prescaled=True)
            for c in self.clients:
                c.apply_step(it)
            packs = [c.pack_buffers() for c in self.clients]
            self.agg.average_(packs, prescaled=True)
            for c, p in zip(self.clients, packs):
                c.unpack_buffers(p)
        else:
            self.agg.average_([c.shared for c in self.clients], prescaled=True)

    def run(self, timing_warmup: int = 0) -> Dict:
        """Runs the remaining rounds.  ``timing_warmup``: the first rounds are excluded
        from the reported wall time (bench)."""
        t0 = time.perf_counter()
        start = self.round
        timed_from = start
        last = start - 1
        self._stop = False
        win = RoundWindow(self._sync)
        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) \
            if (self.device.type == "cuda" and timing_warmup) else None
        kmax = self.rounds_per_replay()
        ends = {self.max_iters - 1}
        if kmax > 1:
            self.prewarm(kmax)
            for c in self.clients:
                ends.update(int(i) for i in np.flatnonzero(c.plan.epoch_end))
                # rounds whose end_round reads the state on the host (round 0's results when
                # num_epochs <= 0, ...): a run must end there, as run_distributed's do
                ends.update(int(i) for i in c.host_heavy_rounds())
        timed_end = start + timing_warmup - 1 if timing_warmup else -1
        covered = start - 1
        with trace_range("rounds"):
            for it in range(self.round, self.max_iters):
                if it > covered:
                    k = 1
                    if kmax > 1:      # (power-of-two runs: few captures, MultiClientRound)
                        k = 1 << ((self._run_end(it, kmax, ends, timed_end) - it + 1).bit_length() - 1)
                    self._round(it, k)
                    covered = it + k - 1
                done = [c.end_round(it) for c in self.clients]
                self._after_round(it, win, done)
                last = it
                if timing_warmup and it == start + timing_warmup - 1:
                    self._sync()
                    t0 = time.perf_counter()
                    if ev is not None:
                        ev[0].record()
                    timed_from = it + 1
                    win.reset()
                if self._stop:
                    break
        if ev is not None:
            ev[1].record()
        self._sync()
        wall = time.perf_counter() - t0
        device_s = ev[0].elapsed_time(ev[1]) * 1e-3 if ev is not None and timed_from > start else None
        n_rounds = last + 1 - timed_from
        docs = sum(int(c.plan.size[timed_from:last + 1].sum()) for c in self.clients) \
            if n_rounds > 0 else 0
        for c in self.clients:
            c.flush()
        self.metrics.write(event="train_end", rounds=n_rounds, wall_s=wall,
                           **self.clients[0].tm.engine_info,
                           docs=docs, docs_per_s=docs / wall if wall and docs else None,
                           ms_per_round=1e3 * wall / max(n_rounds, 1))
        with trace_range("finish"):
            self.finish()
        return {"rounds": self.round, "timed_rounds": n_rounds, "wall_s": wall, "docs": docs,
                "device_s": device_s}

    def _after_round(self, it: int, win: RoundWindow, done: List[bool]):
        self.round = it + 1
        win.add(sum(int(c.plan.size[it]) for c in self.clients))
        if self.metrics_every and self.round % self.metrics_every == 0:
            self._window_metrics(win, it)
        if self.checkpoint_dir and self.checkpoint_every and self.round % self.checkpoint_every == 0:
            with trace_range("checkpoint"):
                for c in self.clients:
                    ckpt.save_client_checkpoint(self.checkpoint_dir, c, self.round)
        if self.stop_at_num_epochs and all(done):
            self.logger.info("-- -- All clients reached num_epochs; stopping at round %d",
                             self.round)
            self._stop = True

    def _window_metrics(self, win: RoundWindow, it: int):
        w = win.close()
        if w is None:
            return
        self.metrics.write(event="window", round=it + 1, **term_window(self.clients, it, w), **w)

    def finish(self):
        for c in self.clients:
            if c.save_path and not c.results_saved:
                c.save_results(c.save_path)
                c.results_saved = True
        if self.save_server:
            self.save_global(server_model_path(self.save_server, self.stamp))

    def save_global(self, path: str):
        """The global model = the averaged state (B4/B5); betas only, like the reference."""
        tm = self.clients[0].tm
        self.logger.info("-- -- Saving global model...")
        save_model_as_npz(path, tm.get_topic_word_distribution(), None, tm.n_components, None)
        return path


# ---------------------------------------------------------------------------
# one process per client (torch.distributed)
# ---------------------------------------------------------------------------
def rehearsal_enabled() -> bool:
    """GFEDNTM_REHEARSE_1GPU=1: every rank on cuda:0 over a gloo process group, with
    the in-step xGMI all-reduce attached -- rehearses the production multi-GPU path
    (same kernels, same IPC protocol; several ranks share the card) on a one-GPU box."""
    return os.environ.get("GFEDNTM_REHEARSE_1GPU", "0") == "1"


class CommError(RuntimeError):
    """A bounded xGMI all-reduce wait timed out: the shared state since is invalid."""


def run_distributed(corpus, params: Dict, model_type: str = "avitm",
                    max_iters: int = 100, backend: str = "auto", data_backend: Optional[str] = None,
                    grads_to_share: Sequence[str] = DEFAULT_GRADS_TO_SHARE, seed: int = 0,
                    save_client: Optional[str] = None, save_server: Optional[str] = None,
                    logger=None, graph: bool = True, log_every: int = 0,
                    stop_at_num_epochs: bool = False, checkpoint_dir: Optional[str] = None,
                    checkpoint_every: int = 0, stamp: Optional[str] = None,
                    bucket_bytes: int = 64 << 20, metrics_path: Optional[str] = None,
                    metrics_every: int = 0, heartbeat_timeout: float = 0.0,
                    agg_mode: str = "params", timing_warmup: int = 0,
                    rehearse_1gpu: Optional[bool] = None, allreduce: Optional[str] = None,
                    round_hook=None, client_ids: Optional[Sequence[int]] = None,
                    keep_round: bool = False, fedavg_wire: str = "fp32") -> Dict:
    """Runs this process's client(s); torch.distributed must be initialised (RANK /
    WORLD_SIZE).  ``corpus`` is this rank's one client (id rank + 1), or a list of client
    corpora with their ids ``client_ids`` -- a contiguous block of a federation of more
    clients than ranks (federation/hierarchical.py assign_clients; the ranks' blocks
    must partition 1..N in rank order).  Rank 0 also plays the coordinator (global
    save).  ``data_backend`` is the process group's backend ('nccl' = RCCL or 'gloo'); a
    separate gloo group carries the control plane.  ``agg_mode`` "params" is the
    reference FedAvg of the shared state after every local step; "grads" all-reduces the
    pre-scaled gradients before one optimizer step on every rank (classic synchronous data
    parallelism; BN statistics averaged; one client per rank).

    Round loop (reference server.py:436-521 + client.py:135-183): the host only
    enqueues work -- one hipGraph replay per round with the FedAvg all-reduce
    captured inside it (fused engine; federation/rank_round.py) -- and never waits for the
    device, except at the rounds where some client does long host work (results /
    snapshot saves, checkpoints, metrics windows).  Those rounds are known to every rank
    up front (:meth:`FederatedClient.host_heavy_rounds`), so all ranks meet there on the
    control plane: no rank's device is left spinning in the in-step xGMI all-reduce while
    a peer's host is busy.  At each such point, every ``GFEDNTM_COMM_POLL`` rounds in
    between (an error word copied behind the enqueued rounds, no sync) and at the end,
    the ranks agree on the all-reduce's error word; a timed-out wait aborts every rank
    with :class:`CommError` (its xGMI resources released) before anything is saved.
    ``heartbeat_timeout`` > 0 adds the control-plane watchdog (parallel/heartbeat.py).

    ``timing_warmup``: the first rounds (after ``start``) are excluded from the
    reported wall time (bench).  ``round_hook(it)`` is called after every round
    (tests inject host stalls with it).  ``GFEDNTM_INJECT_STALL=rank:round:seconds``
    injects one such stall from the environment (failure-injection tests of processes
    this code does not start itself, e.g. bench.py's ranks).

    Cross-rank state check (parallel/digest.py): every ``GFEDNTM_DIGEST_EVERY`` rounds
    (default: the poll interval) each rank digests its clients' shared state behind the
    round (two small kernels + an 8-byte copy, no sync) and the ranks compare the digests
    at the next interval; at the start (W0), at every aligned round and at the end they
    compare synchronously.  A mismatch -- replicas that silently diverged although every
    wait returned -- stops every rank with :class:`CommError`.
    ``GFEDNTM_INJECT_CORRUPT=rank:round`` flips one word of that rank's shared state after
    every round from ``round`` on (a persistent data-plane fault; a one-off divergence is
    re-averaged by the next all-reduce and leaves the replicas equal again).

    ``fedavg_wire``: "fp32" (default; the reference's averaging) or "bf16delta" -- the
    opt-in reduced-byte FedAvg: each rank sends its pre-scaled state's departure from the
    last averaged state in bf16 (half the bytes over xGMI), summed in fp32
    (parallel/aggregator.py, csrc/comm.hip gfk_xgmi_allreduce_bf16d).

    ``keep_round``: leave the rank's data plane attached after the run (the caller closes
    ``out["round"]``; bench.py times the bare engine loop on it); by default it is
    released before returning, on success or error."""
    import torch.distributed as dist
    from .hierarchical import agree_client_map
    from .rank_round import MultiClientRound, SingleClientRound
    logger = logger or logging.getLogger("gfedntm_amd.federation")
    rank, world = dist.get_rank(), dist.get_world_size()
    corpora = [corpus] if isinstance(corpus, ClientCorpus) else list(corpus)
    if client_ids is None:
        if len(corpora) != 1:
            raise ValueError("several client corpora need their client_ids")
        client_ids = [rank + 1]
    client_ids = [int(i) for i in client_ids]
    if len(corpora) != len(client_ids) or not corpora:
        raise ValueError("one corpus per local client id")
    if len(corpora) > 1 and agg_mode != "params":
        raise ValueError("agg_mode 'grads' runs one client per rank")
    inj = os.environ.get("GFEDNTM_INJECT_STALL")
    if inj and round_hook is None:
        r_s, it_s, sec_s = inj.split(":")
        if int(r_s) == rank:
            def round_hook(it, _at=int(it_s), _sec=float(sec_s)):
                if it == _at:
                    time.sleep(_sec)
    data_backend = data_backend or dist.get_backend()
    rehearse = rehearsal_enabled() if rehearse_1gpu is None else bool(rehearse_1gpu)
    ctrl = dist.new_group(backend="gloo") if data_backend != "gloo" else None
    on_gpu_plane = data_backend == "nccl" or rehearse
    if on_gpu_plane:
        device = torch.device("cuda", torch.cuda.current_device())
    else:
        device = torch.device("cpu")
    stamp = stamp or datetime.datetime.now().strftime("%Y%m%d")
    metrics = MetricsWriter(metrics_path)
    hb = None
    if heartbeat_timeout and world > 1:
        from ..parallel.heartbeat import Heartbeat
        hb = Heartbeat(rank, world, timeout=heartbeat_timeout,
                       interval=max(0.5, min(5.0, heartbeat_timeout / 10))).start()
    # ---- stage 1: client map, vocabulary union, weights (control plane) ----
    with trace_range("consensus"):
        cmap = agree_client_map(client_ids, world, group=ctrl)
        gathered: List = [None] * world
        dist.all_gather_object(gathered, [(c.local_terms(), c.n_docs) for c in corpora],
                               group=ctrl)
    every = [x for g in gathered for x in g]              # client-id order
    terms = union_vocabulary([t for t, _ in every])
    vocab = vocabulary_dict(terms)
    weights = fedavg_weights([nd for _, nd in every])
    if rank == 0:
        logger.info("-- -- Global vocabulary agreed: %d terms from %d clients%s", len(terms),
                    len(every), f" on {world} ranks" if len(every) != world else "")
    clients: List[FederatedClient] = []
    for k, (cid, corp) in enumerate(zip(client_ids, corpora)):
        ds = build_dataset(model_type, corp, vocab, terms)
        tm = make_topic_model(model_type, params, len(terms), device, backend, grads_to_share,
                              seed=seed, logger=logger)
        if k == 0:
            # identical W0 on every client: the flat buffer holds every float parameter and buffer
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
                            epoch_snapshots=(model_type in CTM_TYPES), agg=agg_mode)
        c.set_fedavg_weight(weights[cid - 1])
        c.ground_truth = corp.ground_truth()
        c.enable_graph(graph and agg_mode == "params")
        clients.append(c)
    # ---- data plane: this rank's round (its clients' steps + the FedAvg) ----
    if len(clients) == 1:
        rr = SingleClientRound(clients[0], world, device, on_gpu_plane, allreduce, agg_mode,
                               bucket_bytes, logger, wire=fedavg_wire)
    else:
        rr = MultiClientRound(clients, world, device, on_gpu_plane, allreduce, graph, logger,
                              wire=fedavg_wire)
    ok = False
    try:
        out = _round_loop(rr, clients, client_ids, cmap, world, rank, device, ctrl, hb, logger,
                          max_iters, stop_at_num_epochs, checkpoint_dir, checkpoint_every,
                          metrics, metrics_every, timing_warmup, round_hook, agg_mode,
                          save_server, stamp)
        ok = True
        return out
    finally:
        if hb is not None:
            hb.stop()
        if not (ok and keep_round):
            rr.close()


def _inject_corrupt(rank: int):
    """GFEDNTM_INJECT_CORRUPT=rank:round -> the first round it applies on this rank."""
    inj = os.environ.get("GFEDNTM_INJECT_CORRUPT")
    if not inj:
        return None
    r_s, it_s = inj.split(":")[:2]
    return int(it_s) if int(r_s) == rank else None


def _flip_word(t: torch.Tensor):
    """Flip the low bit of the middle word of a shared state (enqueued on the stream)."""
    j = t.numel() // 2
    t.view(torch.int32)[j:j + 1].bitwise_xor_(1)


def _round_loop(rr, clients, client_ids, cmap, world, rank, device, ctrl, hb, logger, max_iters,
                stop_at_num_epochs, checkpoint_dir, checkpoint_every, metrics, metrics_every,
                timing_warmup, round_hook, agg_mode, save_server, stamp) -> Dict:
    import torch.distributed as dist
    from ..parallel.digest import DigestProbe, compare
    start = 0
    # loss / KL / RL histories for the metrics windows and the per-minibatch log line
    record_terms(clients, bool(metrics_every or any(c.log_every for c in clients)))
    if checkpoint_dir:
        starts = {ckpt.load_client_checkpoint(checkpoint_dir, c) for c in clients}
        if len(starts) != 1:
            raise RuntimeError(f"inconsistent client checkpoints on rank {rank}: {sorted(starts)}")
        start = starts.pop()
        rounds = [None] * world
        dist.all_gather_object(rounds, start, group=ctrl)
        if len(set(rounds)) != 1:
            raise RuntimeError(f"inconsistent client checkpoints: rounds {rounds}")
        rr.resync_reference()            # bf16delta: the loaded state is the last average
    # ---- rounds where every rank meets (some client does long host work after them)
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

    def fail(err: int, where: str):
        if os.environ.get("GFEDNTM_COMM_DEBUG") == "1":
            logger.warning("rank %d xGMI state: %s", rank, rr.debug())
        # (the IPC mappings / step graph are released by run_distributed's finally)
        raise CommError(f"rank {rank}: an xGMI all-reduce wait timed out before {where} "
                        f"(error {err}); the shared state is invalid -- resume from the last "
                        "round checkpoint")

    # ---- cross-rank digests of the shared state (parallel/digest.py) ----
    poll_default = os.environ.get("GFEDNTM_COMM_POLL", "512")
    digest_every = (int(os.environ.get("GFEDNTM_DIGEST_EVERY", poll_default))
                    if world > 1 and agg_mode == "params" else 0)
    probe = DigestProbe([c.shared for c in clients]) if digest_every else None
    corrupt_from = _inject_corrupt(rank)
    dstats = {"checked": 0, "last": None}

    def digest_check(res):
        """All-gather every rank's (round, digests) and agree: raise on a divergence."""
        if res is None:
            return
        per_rank: List = [None] * world
        dist.all_gather_object(per_rank, res, group=ctrl)
        why = compare(per_rank, rank)
        if why is not None:
            logger.error("rank %d: %s", rank, why)
            raise CommError(f"rank {rank}: {why}; the shared state is invalid -- resume from "
                            "the last round checkpoint")
        dstats["checked"] += 1
        dstats["last"] = (per_rank[0][0], f"{per_rank[0][1][0]:016x}")

    def digest_now(it: int):
        """Synchronous digest of round ``it`` (the device must be synchronised)."""
        if probe is None:
            return
        digest_check(probe.result())      # a pending asynchronous one first
        probe.take(it)
        digest_check(probe.result())

    def check_comm(where: str):
        """Agree on the xGMI error word across ranks (synchronises the device)."""
        flag = torch.tensor([int(rr.error())], dtype=torch.int64)
        dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=ctrl)
        if int(flag.item()):
            fail(int(flag.item()), where)

    # a timed-out xGMI wait is also caught between the aligned rounds: every poll_every
    # rounds each rank reads the error word copied behind its enqueued rounds (no device
    # sync) and the ranks agree on it over the control plane, so a run fails within about
    # two poll intervals of the timeout instead of training on for the whole run
    poll_every = int(os.environ.get("GFEDNTM_COMM_POLL", "512")) if rr.xgmi else 0

    def poll_comm(it: int):
        flag = torch.tensor([int(rr.error_poll())], dtype=torch.int64)
        dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=ctrl)
        if int(flag.item()):
            fail(int(flag.item()), f"round {it + 1}")
        rr.error_async()

    def meet(where: str):
        sync()
        check_comm(where)
        dist.barrier(group=ctrl)

    dist.barrier(group=ctrl)
    if probe is not None:
        sync()
        digest_now(start - 1)            # identical W0 (or resumed state) on every rank
    # GFEDNTM_COMM_DEBUG=1: the first rounds synchronised one by one, with their times and
    # the xGMI error word (which round a timed-out wait happened in, and the ranks' skew)
    debug_comm = os.environ.get("GFEDNTM_COMM_DEBUG") == "1" and rr.xgmi
    t_dbg0 = time.perf_counter()
    win = RoundWindow(sync)
    # device time of the timed rounds: events on the round stream around them (the host
    # wall clock below brackets the same rounds with a sync + barrier)
    ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) \
        if (device.type == "cuda" and timing_warmup) else None
    t0 = time.perf_counter()
    timed_from = start
    last = start - 1
    # several rounds per graph replay (MultiClientRound.rounds_per_replay): a run of rounds
    # ends at every round after which the host needs the state -- the aligned / epoch-end
    # rounds, the warmup, poll, digest, metrics and checkpoint boundaries, the last round
    # (and never with a round hook, an injected corruption or the comm debug log)
    kmax = getattr(rr, "rounds_per_replay", lambda: 1)()
    if round_hook is not None or corrupt_from is not None or debug_comm:
        kmax = 1
    ends = set(align) | {stop_after}
    if kmax > 1:
        for c in clients:
            ends.update(int(i) for i in np.flatnonzero(c.plan.epoch_end))
        if timing_warmup:
            ends.add(start + timing_warmup - 1)

    def run_end(it: int) -> int:
        r = it
        while r < it + kmax - 1 and r not in ends:
            n1 = r + 1
            if ((poll_every and n1 % poll_every == 0) or (digest_every and n1 % digest_every == 0)
                    or (metrics_every and n1 % metrics_every == 0)
                    or (checkpoint_dir and checkpoint_every and n1 % checkpoint_every == 0)):
                break
            r += 1
        return r

    if kmax > 1 and hasattr(rr, "prewarm"):
        rr.prewarm(kmax)              # every k-round graph captured before the first round
    covered = start - 1
    with trace_range("rounds"):
        for it in range(start, stop_after + 1):
            if hb is not None:
                hb.mark(it, 0)
            if it > covered:
                # (a power of two: at most log2(kmax) + 1 graphs are ever captured -- a
                # capture inside the timed rounds costs milliseconds)
                k = 1 << ((run_end(it) - it + 1).bit_length() - 1) if kmax > 1 else 1
                if k > 1:
                    rr.step(it, hb, k)
                else:
                    rr.step(it, hb)
                covered = it + k - 1
            elif hb is not None:
                hb.mark(it, 1)
            if corrupt_from is not None and it >= corrupt_from:
                _flip_word(clients[0].shared)
            if debug_comm and it < start + 16:
                t_dbg = time.perf_counter()
                sync()
                logger.warning("rank %d round %d: enqueued at %.3f s, done at %.3f s, xGMI "
                               "error %d", rank, it, t_dbg - t_dbg0, time.perf_counter() - t_dbg0,
                               rr.error())
            heavy = it in align
            if heavy:
                # validate the state before anything is exported
                sync()
                check_comm(f"the host work of round {it}")
                digest_now(it)
                if hb is not None:
                    hb.busy(True)
            for c in clients:
                c.end_round(it)
            last = it
            if heavy:
                if hb is not None:
                    hb.busy(False)
                dist.barrier(group=ctrl)
            if poll_every and (it + 1) % poll_every == 0 and it != stop_after:
                poll_comm(it)
            if digest_every and (it + 1) % digest_every == 0 and it != stop_after and not heavy:
                # the previous interval's digest (landed long ago), then this round's
                digest_check(probe.result())
                probe.take(it)
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
                metrics.write(event="window", rank=rank, round=it + 1,
                              **term_window(clients, it, w or {}), **(w or {}))
            if checkpoint_dir and checkpoint_every and (it + 1) % checkpoint_every == 0:
                with trace_range("checkpoint"):
                    meet(f"checkpoint {it + 1}")
                    if hb is not None:
                        hb.busy(True)
                    for c in clients:
                        ckpt.save_client_checkpoint(checkpoint_dir, c, it + 1)
                    if hb is not None:
                        hb.busy(False)
                    dist.barrier(group=ctrl)
    if ev is not None:
        ev[1].record()
    sync()
    wall = time.perf_counter() - t0
    device_s = ev[0].elapsed_time(ev[1]) * 1e-3 if ev is not None and timed_from > start else None
    check_comm("the end of training")
    digest_now(last)
    for c in clients:
        c.flush()
    n_rounds = last + 1 - timed_from
    docs = sum(int(c.plan.size[timed_from: last + 1].sum()) for c in clients) if n_rounds > 0 else 0
    metrics.write(event="train_end", rank=rank, clients=list(client_ids), rounds=n_rounds,
                  **clients[0].tm.engine_info,
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
    return {"rounds": last + 1, "timed_rounds": n_rounds, "wall_s": wall, "docs": docs,
            "device_s": device_s, "client": clients[0], "clients": clients, "client_map": cmap,
            "allreduce": rr.method, "attach": rr.attach, "round": rr,
            "digests": dict(dstats, every=digest_every)}
