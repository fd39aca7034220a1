"""Local-step engines.

An engine owns one client's model state (flat buffer + optimizer state) and
runs *one local minibatch step* = zero_grad -> forward -> loss -> backward ->
optimizer step (reference federated_avitm.py:51-83, federated_ctm.py:50-114).

* :class:`TorchEngine` -- stock PyTorch ops; the numerical oracle and the CPU
  path (tests, gloo federation, any solver / activation / model variant).
* :class:`gfedntm_amd.ops.engine.FusedEngine` -- hand-written CDNA4 HIP
  kernels + fused multi-tensor Adam + hipGraph replay (MI355X training path).

Both read minibatches from a device-resident CSR shard through a
:class:`~gfedntm_amd.data.bow.BatchPlan`, and both record the loss of step s
into ``loss_hist[s]`` on device, so the host only synchronizes when it logs.
"""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch
from torch import optim

from ..data.bow import BatchPlan, DeviceCSR
from ..utils.flat import FlatState
from .networks import kl_terms, reconstruction_terms


def make_optimizer(params, solver: str, lr: float, momentum: float):
    """Reference optimizer table (avitm.py:141-153, ctm.py:158-168)."""
    if solver == "adam":
        return optim.Adam(params, lr=lr, betas=(momentum, 0.99))
    if solver == "sgd":
        return optim.SGD(params, lr=lr, momentum=momentum)
    if solver == "adagrad":
        return optim.Adagrad(params, lr=lr)
    if solver == "adadelta":
        return optim.Adadelta(params, lr=lr)
    if solver == "rmsprop":
        return optim.RMSprop(params, lr=lr, momentum=momentum)
    raise ValueError("solver must be 'adam', 'adadelta', 'sgd', 'rmsprop' or 'adagrad'")


class EngineBase:
    kind = "avitm"   # or "ctm"

    def __init__(self, model, flat: FlatState, loss_weight_beta: float = 1.0):
        self.model = model
        self.flat = flat
        self.beta_weight = float(loss_weight_beta)
        self.data: Optional[DeviceCSR] = None
        self.plan: Optional[BatchPlan] = None
        self.loss_hist: Optional[torch.Tensor] = None
        # per-step mean KL / reconstruction terms (metrics windows, the per-minibatch log):
        # the fused kernels fill them only while record_terms(True) is set
        self.kl_hist: Optional[torch.Tensor] = None
        self.rl_hist: Optional[torch.Tensor] = None
        self.terms_on = False

    @property
    def device(self):
        return self.flat.buffer.device

    def bind_data(self, data: DeviceCSR, plan: BatchPlan):
        self.data, self.plan = data, plan
        self.loss_hist = torch.zeros(plan.n_steps, dtype=torch.float32, device=self.device)
        self.kl_hist = torch.zeros(plan.n_steps, dtype=torch.float32, device=self.device)
        self.rl_hist = torch.zeros(plan.n_steps, dtype=torch.float32, device=self.device)

    def record_terms(self, on: bool = True):
        """Keep the per-step mean KL and reconstruction terms in ``kl_hist`` / ``rl_hist``
        (reference federated_avitm.py:109 logs the minibatch loss; SURVEY 5.5 asks for the
        split).  Host-cheap for the torch engine; a flag of the fused kernels."""
        self.terms_on = bool(on)

    def term_means(self, s0: int, s1: int):
        """(loss, KL, RL) means over steps [s0, s1) (None for terms not recorded)."""
        if self.loss_hist is None or s1 <= s0:
            return None, None, None
        loss = float(self.loss_hist[s0:s1].mean())
        if not self.terms_on:
            return loss, None, None
        return loss, float(self.kl_hist[s0:s1].mean()), float(self.rl_hist[s0:s1].mean())

    def step(self, s: int) -> torch.Tensor:
        raise NotImplementedError

    # ---- split step for gradient aggregation (classic synchronous data parallelism):
    # compute_grads leaves this step's gradients in a flat buffer with the parameter
    # layout (grad_buffer), the transport averages its shared prefix, apply_grads runs
    # the optimizer on the averaged gradients.
    def compute_grads(self, s: int) -> torch.Tensor:
        raise NotImplementedError

    def apply_grads(self, s: int):
        raise NotImplementedError

    @property
    def grad_shared(self) -> torch.Tensor:
        return self.grad_buffer[: self.flat.n_shared]

    def optimizer_state_dict(self):
        return self.optimizer.state_dict()

    def load_optimizer_state_dict(self, sd):
        self.optimizer.load_state_dict(sd)

    # the part of the state that is averaged every round
    @property
    def shared(self) -> torch.Tensor:
        return self.flat.shared


class TorchEngine(EngineBase):
    """Reference-exact local step on stock PyTorch ops."""

    def __init__(self, model, flat: FlatState, solver="adam", lr=2e-3, momentum=0.99,
                 reduce_on_plateau=False, loss_weight_beta: float = 1.0, kind: str = "avitm"):
        super().__init__(model, flat, loss_weight_beta)
        self.kind = kind
        self.optimizer = make_optimizer(model.parameters(), solver, lr, momentum)
        self.scheduler = (optim.lr_scheduler.ReduceLROnPlateau(self.optimizer, patience=10)
                          if reduce_on_plateau else None)

    # ---- per-client random streams: dropout / reparameterisation noise drawn from the
    # engine's own generator state instead of the process-global one, so a client's
    # noise does not depend on how many other clients share its process (LocalFederation
    # vs one or several clients per rank)
    _rng_cpu = None
    _rng_dev = None

    def own_rng(self, seed: int):
        self._rng_cpu = torch.Generator().manual_seed(int(seed)).get_state()
        if self.device.type == "cuda":
            self._rng_dev = torch.Generator(device=self.device).manual_seed(int(seed)).get_state()

    def rng_state(self):
        return None if self._rng_cpu is None else (self._rng_cpu, self._rng_dev)

    def set_rng_state(self, st):
        if st is not None:
            self._rng_cpu, self._rng_dev = st

    def _run_with_rng(self, fn):
        if self._rng_cpu is None:
            return fn()
        cuda = self.device.type == "cuda"
        with torch.random.fork_rng(devices=[self.device] if cuda else []):
            torch.set_rng_state(self._rng_cpu)
            if cuda:
                torch.cuda.set_rng_state(self._rng_dev, self.device)
            out = fn()
            self._rng_cpu = torch.get_rng_state()
            if cuda:
                self._rng_dev = torch.cuda.get_rng_state(self.device)
        return out

    def _batch(self, s: int):
        ids = torch.from_numpy(self.plan.batch(s).astype(np.int64)).to(self.device)
        x = self.data.dense_rows(ids)
        ctx = self.data.contextual[ids] if self.data.contextual is not None else None
        lab = self.data.labels[ids] if self.data.labels is not None else None
        return x, ctx, lab

    def loss_on(self, x, ctx=None, labels=None):
        """Forward + loss of one minibatch (reference avitm.py:168-229 / ctm.py:182-296)."""
        m = self.model
        if self.kind == "ctm":
            pm, pv, mu, var, logvar, wd, est = m(x, ctx, labels)
        else:
            pm, pv, mu, var, logvar, wd = m(x)
            est = None
        kl = kl_terms(pm, pv, mu, var, logvar, m.n_components)
        rl = reconstruction_terms(x, wd)
        self._terms = (kl.detach(), rl.detach())
        loss = (self.beta_weight * kl + rl).sum()
        if labels is not None and est is not None:
            loss = loss + torch.nn.functional.cross_entropy(est, torch.argmax(labels, 1))
        return loss

    def _record(self, s: int, loss: torch.Tensor):
        self.loss_hist[s] = loss.detach()
        if self.terms_on:
            kl, rl = self._terms
            self.kl_hist[s] = kl.mean()
            self.rl_hist[s] = rl.mean()

    def step(self, s: int) -> torch.Tensor:
        return self._run_with_rng(lambda: self._step(s))

    def _step(self, s: int) -> torch.Tensor:
        self.model.train()
        x, ctx, lab = self._batch(s)
        self.model.zero_grad()
        loss = self.loss_on(x, ctx, lab)
        loss.backward()
        self.optimizer.step()
        self._record(s, loss)
        return loss.detach()

    @property
    def grad_buffer(self) -> torch.Tensor:
        if getattr(self, "_grad_buf", None) is None:
            self._grad_buf = torch.zeros_like(self.flat.buffer)
        return self._grad_buf

    def compute_grads(self, s: int) -> torch.Tensor:
        return self._run_with_rng(lambda: self._compute_grads(s))

    def _compute_grads(self, s: int) -> torch.Tensor:
        self.model.train()
        x, ctx, lab = self._batch(s)
        self.model.zero_grad()
        loss = self.loss_on(x, ctx, lab)
        loss.backward()
        g = self.grad_buffer
        g.zero_()
        for k, p in self.model.named_parameters():
            if p.grad is not None:
                self.flat.view_like(g, k).copy_(p.grad)
        self._record(s, loss)
        return loss.detach()

    def apply_grads(self, s: int):
        g = self.grad_buffer
        for k, p in self.model.named_parameters():
            if p.grad is not None:
                p.grad.copy_(self.flat.view_like(g, k))
        self.optimizer.step()
