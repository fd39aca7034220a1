"""One federation client: local shard + model + the reference round bookkeeping.

Reference: src/models/federated/federated_avitm.py:51-147 (``train_mb_delta`` /
``deltaUpdateFit``), federated_ctm.py:59-188, federated_model.py:57-197.

Per round (``local_step`` then, after the aggregation, ``end_round``):
  * one local minibatch step -- zero_grad, forward, loss, backward, optimizer
    (the engine; on MI355X one hipGraph replay of the fused HIP step);
  * the sample-weighted average of the shared state replaces the local copy
    (done by the transport: in-process sum, RCCL all-reduce or gRPC);
  * bookkeeping exactly like the reference: current minibatch / epoch, samples
    processed, the epoch summary line, best components, and the results save
    once ``num_epochs`` is reached.

``agg="grads"`` (classic synchronous data parallelism, not the reference
semantics): ``local_step`` leaves the step's gradients in the engine's flat
gradient buffer pre-scaled by w_i, the transport sums their shared prefix,
``apply_step`` runs the optimizer on the averaged gradients -- the replicas stay
identical -- and the batch-norm running statistics are averaged separately
(``pack_buffers`` / ``unpack_buffers``).

Differences by design: the per-minibatch loss line needs the loss on the host,
which would force a device sync every round, so it is logged every
``log_every`` rounds (0 = never).  The epoch summary never stalls the device:
at an epoch end the epoch's loss sum is reduced on device and copied into
pinned host memory behind an event; the line is emitted (with the reference
arithmetic) by :meth:`poll` once the event has completed, or by :meth:`flush`.  The results are saved once when
``num_epochs`` is reached (the reference re-runs inference and re-saves on every
later round, B16) and, optionally, the client stops (``stop_at_num_epochs``).
"""
from __future__ import annotations

import datetime
import logging
from typing import List, Optional

import numpy as np
import torch

from ..data.bow import BatchPlan
from ..eval.export import postprocess_thetas, save_model_as_npz


class FederatedClient:
    def __init__(self, client_id: int, tm, dataset, max_iters: int, logger=None, seed: int = 0,
                 save_path: Optional[str] = None, log_every: int = 0, n_samples: int = 20,
                 epoch_snapshots: bool = False, agg: str = "params"):
        if agg not in ("params", "grads"):
            raise ValueError("agg must be 'params' (FedAvg) or 'grads' (gradient all-reduce)")
        self.agg = agg
        self.id = client_id
        self.tm = tm
        self.dataset = dataset
        self.logger = logger or logging.getLogger(f"gfedntm_amd.client{client_id}")
        self.save_path = save_path
        self.log_every = log_every
        self.n_samples = n_samples
        self.epoch_snapshots = epoch_snapshots
        tm.train_data = dataset
        self.data = tm.device_data(dataset)
        self.n_docs = self.data.n_docs
        self.max_iters = max_iters
        self.plan = BatchPlan.build(self.n_docs, tm.batch_size, max_iters, seed=seed)
        if agg == "grads" and tm.backend == "fused":
            from ..ops.engine import UPDATE_GRAD
            tm.engine.set_update_mode(UPDATE_GRAD)
        tm.engine.bind_data(self.data, self.plan)
        if hasattr(tm.engine, "own_rng"):     # PyTorch engine: a per-client noise stream
            tm.engine.own_rng(seed)
        tm.model.train()
        self.weight: Optional[float] = None
        # synthetic ground truth (doc-topic, topic-word over the generator vocabulary):
        # scored at every results save, like the reference's evaluate_synthetic_model
        self.ground_truth = None
        self.synthetic_eval: Optional[dict] = None
        # reference bookkeeping
        self.current_mb = 0
        self.current_epoch = 0
        self.samples_processed = 0
        self.train_loss = 0.0
        self.epoch_first_step = 0
        self.results_saved = False
        tm.best_components = tm.model.beta       # the reference keeps a live reference
        # epoch summaries in flight: (epoch index, samples processed, pinned loss, event).
        # The pinned ring, the events and the reduction kernel are set up here, not at
        # the first epoch end, so no one-time cost lands inside the round loop.
        self._pending: List[tuple] = []
        self._pinned = None
        self._events: List = []
        self._slot = 0
        hist = tm.engine.loss_hist
        if hist.device.type == "cuda":
            self._pinned = torch.zeros(64, dtype=torch.float32, pin_memory=True)
            self._events = [torch.cuda.Event() for _ in range(self._pinned.numel())]
            self._pinned[:1].copy_(hist[:1].sum().view(1), non_blocking=True)
            torch.cuda.synchronize(hist.device)

    # ------------------------------------------------------------------ state
    @property
    def shared(self) -> torch.Tensor:
        return self.tm.flat.shared

    @property
    def fused(self) -> bool:
        return self.tm.backend == "fused"

    def set_fedavg_weight(self, w: float):
        """Pre-scale the shared state by w_i = n_i / sum n after every local step, so the
        aggregation is a plain sum (fused engine: inside the update kernels)."""
        self.weight = float(w)
        if self.fused and self.agg == "params":
            self.tm.engine.set_fedavg_scale(self.weight)

    def enable_graph(self, on: bool = True):
        if self.fused:
            self.tm.engine.enable_graph(on)

    # ------------------------------------------------------------------ round
    def local_step(self, it: int):
        if self.agg == "grads":
            self.tm.engine.compute_grads(it)
            if self.weight is not None:
                self.shared_grads.mul_(self.weight)
            return
        self.tm.engine.step(it)
        if self.weight is not None and not self.fused:
            self.shared.mul_(self.weight)

    # ---- gradient aggregation (agg="grads") ----
    @property
    def shared_grads(self) -> torch.Tensor:
        return self.tm.engine.grad_shared

    def apply_step(self, it: int):
        """Optimizer step on the aggregated gradients."""
        self.tm.engine.apply_grads(it)

    def pack_buffers(self) -> torch.Tensor:
        """The shared batch-norm running statistics, pre-scaled by w_i, in one buffer."""
        flat = self.tm.flat
        parts = [flat.buffer[s.offset: s.offset + s.numel] for s in flat.shared_buffer_slots()]
        if not parts:
            return torch.zeros(0, device=flat.buffer.device)
        out = torch.cat(parts)
        if self.weight is not None:
            out.mul_(self.weight)
        return out

    def unpack_buffers(self, packed: torch.Tensor):
        o = 0
        flat = self.tm.flat
        for s in flat.shared_buffer_slots():
            flat.buffer[s.offset: s.offset + s.numel].copy_(packed[o: o + s.numel])
            o += s.numel

    def end_round(self, it: int) -> bool:
        """Bookkeeping after the aggregated state was loaded; True when this client has
        reached ``num_epochs`` (results saved)."""
        nb = int(self.plan.size[it])
        self.samples_processed += nb
        if self.log_every and it % self.log_every == 0:
            # the reference line (federated_avitm.py:109), then the loss's KL / RL split
            e = self.tm.engine
            loss = float(e.loss_hist[it].item())
            if e.terms_on:
                self.logger.info("-- -- Minibatch %d loss %s / samples processes %d / KL %.6g RL %.6g",
                                 self.current_mb, loss, self.samples_processed,
                                 float(e.kl_hist[it].item()), float(e.rl_hist[it].item()))
            else:
                self.logger.info("-- -- Minibatch %d loss %s / samples processes %d", self.current_mb,
                                 loss, self.samples_processed)
        self.current_mb += 1
        if bool(self.plan.epoch_end[it]):
            self._queue_epoch_summary(self.epoch_first_step, it)
            if self.epoch_snapshots and self.save_path:
                self.flush()
                self.save_results(self.save_path.replace(".npz", f"_epoch_{self.current_epoch}.npz"))
            self.current_epoch += 1
            self.current_mb = 0
            self.epoch_first_step = it + 1
        if self.current_epoch >= self.tm.num_epochs and not self.results_saved:
            self.flush()
            self.logger.info("Epoch end reached")
            if self.save_path:
                self.save_results(self.save_path)
            self.results_saved = True
        self.poll()
        return self.results_saved

    # ---- asynchronous epoch summaries
    def _queue_epoch_summary(self, first: int, last: int):
        hist = self.tm.engine.loss_hist
        if hist.device.type != "cuda":
            self._pending.append((self.current_epoch, self.samples_processed,
                                  float(hist[first: last + 1].sum()), None))
            self.poll()
            return
        # a ring of pinned slots: more epochs than slots can't be in flight at once
        if len(self._pending) >= self._pinned.numel():
            self.flush()
        slot = self._slot
        self._slot = (slot + 1) % self._pinned.numel()
        dst = self._pinned[slot: slot + 1]
        dst.copy_(hist[first: last + 1].sum().view(1), non_blocking=True)
        ev = self._events[slot]
        ev.record()
        self._pending.append((self.current_epoch, self.samples_processed, dst, ev))

    def _emit(self, epoch: int, samples: int, epoch_loss: float):
        # reference arithmetic: train_loss accumulates and is divided by the running
        # sample count at every epoch end (federated_avitm.py:107-119)
        self.train_loss += epoch_loss
        self.train_loss /= samples
        self.logger.info("Epoch: [%d/%d]\tSamples: [%d/%d]\tTrain Loss: %s\tTime: %s",
                         epoch + 1, self.tm.num_epochs, samples,
                         self.n_docs * self.tm.num_epochs, self.train_loss,
                         datetime.datetime.now())
        if epoch == 0 or self.train_loss < self.tm.best_loss_train:
            self.tm.best_loss_train = min(self.tm.best_loss_train, self.train_loss)

    def poll(self, block: bool = False):
        """Emit the epoch summaries whose device reduction has landed (in order)."""
        while self._pending:
            epoch, samples, val, ev = self._pending[0]
            if ev is not None:
                if not block and not ev.query():
                    return
                ev.synchronize()
                val = float(val.item())
            self._pending.pop(0)
            self._emit(epoch, samples, float(val))

    def flush(self):
        """Emit every pending epoch summary (waits for the device)."""
        self.poll(block=True)

    def host_heavy_rounds(self) -> List[int]:
        """Rounds after which this client does long host-side work (results / epoch
        snapshot saves: full-shard inference + npz write).  A pure function of the
        shard size, batch size and num_epochs, so every rank can agree on them up
        front (the distributed runner aligns all ranks there)."""
        if not self.save_path:
            return []
        ends = [int(i) for i in np.flatnonzero(self.plan.epoch_end)]
        out = set(ends) if self.epoch_snapshots else set()
        ne = int(self.tm.num_epochs)
        if not self.results_saved:
            if ne <= 0:
                out.add(0)
            elif len(ends) >= ne:
                out.add(ends[ne - 1])
        return sorted(out)

    def done_round(self) -> Optional[int]:
        """The round at whose end this client reaches ``num_epochs`` (None: never
        within the plan)."""
        ne = int(self.tm.num_epochs)
        if ne <= 0:
            return 0
        ends = np.flatnonzero(self.plan.epoch_end)
        return int(ends[ne - 1]) if len(ends) >= ne else None

    # ------------------------------------------------------------------ results
    def results(self):
        """(betas, thetas, topics) as the reference ``get_results_model`` computes them."""
        tm = self.tm
        topics = tm.get_topics(10)
        thetas = postprocess_thetas(tm.get_doc_topic_distribution(self.dataset, self.n_samples))
        betas = tm.get_topic_word_distribution()
        return betas, thetas, topics

    def save_results(self, path: str) -> str:
        self.logger.info("-- -- Saving model at %s ", path)
        betas, thetas, topics = self.results()
        was_training = self.tm.model.training
        save_model_as_npz(path, betas, thetas, self.tm.n_components, topics)
        self.tm.model.train(was_training)
        if self.ground_truth is not None:
            self.evaluate_synthetic(betas, thetas)
        return path

    def evaluate_synthetic(self, betas: np.ndarray, thetas: np.ndarray) -> dict:
        """TSS / DSS of this client's model against the generator's ground truth, logged
        with the reference's lines (federated_avitm.py:152-193 evaluate_synthetic_model):
        the learned topic-word matrix re-indexed onto the generator vocabulary ('wd<j>' ->
        column j, auxiliary_functions.py:441-483), TSS = sum over ground-truth topics of
        the best Bhattacharyya coefficient, DSS = mean |sqrt(theta) sqrt(theta)^T
        difference| over this client's documents."""
        from ..eval.metrics import betas_to_ground_truth_vocab, dss, tss
        gt_thetas, gt_betas = self.ground_truth
        id2token = getattr(self.dataset, "idx2token", None) or \
            {i: t for i, t in enumerate(getattr(self.tm, "id2token", {}) or {})}
        b = betas_to_ground_truth_vocab(np.asarray(betas), id2token, gt_betas.shape[1])
        th = thetas.toarray() if hasattr(thetas, "toarray") else np.asarray(thetas)
        t_score = tss(b, gt_betas)
        d_score = dss(gt_thetas[: th.shape[0]], th)
        self.logger.info("-- -- Tópicos (equivalentes) evaluados correctamente: %s", t_score)
        self.logger.info("-- -- Difference in evaluation of doc similarity: %s", d_score)
        self.synthetic_eval = {"tss": float(t_score), "dss": float(d_score)}
        return self.synthetic_eval

    def loss_history(self) -> np.ndarray:
        return self.tm.engine.loss_hist.detach().cpu().numpy()
