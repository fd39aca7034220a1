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
``log_every`` rounds (0 = never); the epoch summary reads the whole epoch's
device-resident loss history with one sync.  The results are saved once when
``num_epochs`` is reached (the reference re-runs inference and re-saves on every
later round, B16) and, optionally, the client stops (``stop_at_num_epochs``).
"""
from __future__ import annotations

import datetime
import logging
from typing import Optional

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
        tm.model.train()
        self.weight: Optional[float] = None
        # reference bookkeeping
        self.current_mb = 0
        self.current_epoch = 0
        self.samples_processed = 0
        self.train_loss = 0.0
        self.epoch_first_step = 0
        self.results_saved = False
        tm.best_components = tm.model.beta       # the reference keeps a live reference

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
            loss = float(self.tm.engine.loss_hist[it].item())
            self.logger.info("-- -- Minibatch %d loss %s / samples processes %d", self.current_mb,
                             loss, self.samples_processed)
        self.current_mb += 1
        if bool(self.plan.epoch_end[it]):
            epoch_loss = float(self.tm.engine.loss_hist[self.epoch_first_step: it + 1].sum().item())
            # reference arithmetic: train_loss accumulates and is divided by the running
            # sample count at every epoch end (federated_avitm.py:107-119)
            self.train_loss += epoch_loss
            self.train_loss /= self.samples_processed
            self.logger.info("Epoch: [%d/%d]\tSamples: [%d/%d]\tTrain Loss: %s\tTime: %s",
                             self.current_epoch + 1, self.tm.num_epochs, self.samples_processed,
                             self.n_docs * self.tm.num_epochs, self.train_loss,
                             datetime.datetime.now())
            if self.current_epoch == 0 or self.train_loss < self.tm.best_loss_train:
                self.tm.best_loss_train = min(self.tm.best_loss_train, self.train_loss)
            if self.epoch_snapshots and self.save_path:
                self.save_results(self.save_path.replace(".npz", f"_epoch_{self.current_epoch}.npz"))
            self.current_epoch += 1
            self.current_mb = 0
            self.epoch_first_step = it + 1
        if self.current_epoch >= self.tm.num_epochs and not self.results_saved:
            self.logger.info("Epoch end reached")
            if self.save_path:
                self.save_results(self.save_path)
            self.results_saved = True
        return self.results_saved

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
        return path

    def loss_history(self) -> np.ndarray:
        return self.tm.engine.loss_hist.detach().cpu().numpy()
