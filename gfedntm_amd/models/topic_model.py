"""Centralized neural-topic-model trainers (AVITM / CTM public API).

Public surface follows the reference classes
(reference src/models/base/pytorchavitm/avitm_network/avitm.py:20-640 and
src/models/base/contextualized_topic_models/ctm_network/ctm.py:20-807):
``fit``, ``_loss``, ``_train_epoch``, ``_validate_epoch``,
``get_doc_topic_distribution``, ``get_predicted_topics``,
``get_topic_word_matrix``, ``get_topic_word_distribution``, ``get_topics``,
``save`` / ``load``; CTM adds ``get_word_distribution_by_topic_id``,
``get_top_documents_per_topic_id``, ``get_most_likely_topic`` and
``get_ldavis_data_format``.

What is different by design:
  * data stays on the device as CSR; an epoch is a device-resident
    :class:`BatchPlan`, not a host DataLoader with ``cpu_count()`` workers;
  * the local step runs on an engine: the fused HIP engine on MI355X
    (``backend='fused'``) or the PyTorch oracle (``backend='torch'``);
  * theta inference evaluates the encoder once per document and draws the
    ``n_samples`` reparameterised samples from it (the reference recomputes the
    whole encoder ``n_samples`` times; in eval mode it is deterministic, so the
    result has the same distribution);
  * ``save`` writes a weights-only checkpoint (state_dict + plain config dict),
    loadable with ``torch.load(weights_only=True)``; ``load`` works
    (reference B10 called a nonexistent ``_init_nn``).
"""
from __future__ import annotations

import datetime
import logging
import os
from collections import defaultdict
from typing import Any, Dict, Optional

import numpy as np
import torch
import torch.nn.functional as F

from ..data.bow import BatchPlan, BOWDataset, CTMDataset, DeviceCSR
from ..utils.flat import FlatState
from .engine import TorchEngine
from .networks import ACTIVATIONS, kl_terms, reconstruction_terms

TRANSPOSED_KEYS = ("inf_net.input_layer.weight",)


def default_device():
    return torch.device("cuda" if torch.cuda.is_available() else "cpu")


class EarlyStopping:
    """Patience-based early stopping on validation loss (reference pytorchtools.py:4-55;
    uses ``inf`` instead of ``np.Inf``, which numpy >= 2 removed -- B15)."""

    def __init__(self, patience=7, verbose=False, delta=0.0, path="checkpoint.pt",
                 trace_func=print):
        self.patience, self.verbose, self.delta = patience, verbose, delta
        self.path, self.trace_func = path, trace_func
        self.counter, self.best_score, self.early_stop = 0, None, False
        self.val_loss_min = float("inf")

    def __call__(self, val_loss, model):
        score = -val_loss
        if self.best_score is None:
            self.best_score = score
            self.save_checkpoint(val_loss, model)
        elif score < self.best_score + self.delta:
            self.counter += 1
            if self.verbose:
                self.trace_func(f"EarlyStopping counter: {self.counter} out of {self.patience}")
            if self.counter >= self.patience:
                self.early_stop = True
        else:
            self.best_score = score
            self.save_checkpoint(val_loss, model)
            self.counter = 0

    def save_checkpoint(self, val_loss, model):
        if self.verbose:
            self.trace_func(f"Validation loss decreased ({self.val_loss_min:.6f} --> "
                            f"{val_loss:.6f}).  Saving model ...")
        if self.path is not None:
            model.save(self.path)
        self.val_loss_min = val_loss


class TopicModelBase:
    """Shared trainer logic; subclasses build the network and batch inputs."""

    kind = "avitm"
    model_dir_prefix = "AVITM"

    def __init__(self, logger=None, input_size: int = 0, n_components: int = 10,
                 model_type: str = "prodLDA", hidden_sizes=(100, 100),
                 activation: str = "softplus", dropout: float = 0.2, learn_priors: bool = True,
                 batch_size: int = 64, lr: float = 2e-3, momentum: float = 0.99,
                 solver: str = "adam", num_epochs: int = 100, reduce_on_plateau: bool = False,
                 topic_prior_mean: float = 0.0, topic_prior_variance=None, num_samples: int = 10,
                 num_data_loader_workers: int = 0, verbose: bool = True,
                 backend: str = "auto", device=None, shared_keys=None, seed: Optional[int] = None,
                 loss_weights: Optional[Dict[str, float]] = None, compat_double_softmax=True,
                 matmul_dtype: str = "fp32", **extra):
        if not (isinstance(input_size, (int, np.integer)) and input_size > 0):
            raise ValueError("input_size must be int > 0")
        if not (isinstance(n_components, (int, np.integer)) and n_components > 0):
            raise ValueError("n_components must be int > 0")
        if model_type.lower() not in ("lda", "prodlda"):
            raise ValueError("model must be 'LDA' or 'prodLDA'")
        if not isinstance(hidden_sizes, tuple):
            raise TypeError("hidden_sizes must be type tuple")
        if activation not in ACTIVATIONS:
            raise ValueError(f"activation must be one of {ACTIVATIONS}")
        if dropout < 0:
            raise ValueError("dropout must be >= 0")
        if not (isinstance(batch_size, int) and batch_size > 0):
            raise ValueError("batch_size must be int > 0")
        if lr <= 0:
            raise ValueError("lr must be > 0")
        if not (isinstance(momentum, float) and 0 < momentum <= 1):
            raise ValueError("momentum must be 0 < float <= 1")
        if solver not in ("adagrad", "adam", "sgd", "adadelta", "rmsprop"):
            raise ValueError("solver must be 'adam', 'adadelta', 'sgd', 'rmsprop' or 'adagrad'")
        if not isinstance(topic_prior_mean, float):
            raise TypeError("topic_prior_mean must be type float")
        self.logger = logger or logging.getLogger("gfedntm_amd")
        self.input_size, self.n_components = int(input_size), int(n_components)
        self.model_type, self.hidden_sizes = model_type, hidden_sizes
        self.activation, self.dropout, self.learn_priors = activation, dropout, learn_priors
        self.batch_size, self.lr, self.momentum, self.solver = batch_size, lr, momentum, solver
        self.num_epochs, self.reduce_on_plateau = num_epochs, reduce_on_plateau
        self.topic_prior_mean, self.topic_prior_variance = topic_prior_mean, topic_prior_variance
        self.num_samples, self.num_data_loader_workers = num_samples, num_data_loader_workers
        self.verbose = verbose
        if matmul_dtype not in ("fp32", "bf16"):
            raise ValueError("matmul_dtype must be 'fp32' or 'bf16'")
        # "bf16": the ProdLDA decoder GEMMs take bf16 operands on the matrix cores (fp32
        # accumulation, fp32 parameters / Adam state / everything else) -- fused engine only
        self.matmul_dtype = matmul_dtype
        self.weights = loss_weights or {"beta": 1}
        self.compat_double_softmax = compat_double_softmax
        self.best_loss_train = float("inf")
        self.model_dir = None
        self.train_data = None
        self.validation_data = None
        self.nn_epoch = None
        self.best_components = None
        self.training_doc_topic_distributions = None
        self.device = torch.device(device) if device is not None else default_device()
        if seed is not None:
            torch.manual_seed(seed)
        self.model = self._build_network(**extra).to(self.device)
        self.backend = self._choose_backend(backend)
        if self.matmul_dtype == "bf16" and self.backend != "fused":
            raise ValueError("matmul_dtype='bf16' runs on the fused HIP engine only")
        self.shared_keys = list(shared_keys) if shared_keys is not None else \
            list(self.model.state_dict().keys())
        self._build_engine()
        self.early_stopping = EarlyStopping(patience=5, verbose=False)
        self._device_data: Dict[int, DeviceCSR] = {}

    # ---------------------------------------------------------------- build
    def _build_network(self, **extra):
        raise NotImplementedError

    backend_fallback_reason = None

    @property
    def engine_info(self) -> dict:
        """Which local-step engine runs this model, and why not the fused one if not."""
        d = {"engine": self.backend}
        plan = getattr(getattr(self, "engine", None), "launch_plan", None)
        if isinstance(plan, str):
            d["plan"] = plan
        if self.backend_fallback_reason:
            d["fused_unavailable"] = self.backend_fallback_reason
        return d

    def _choose_backend(self, backend: str) -> str:
        if backend == "auto":
            from ..ops import engine as fused
            from ..ops import native
            if self.device.type != "cuda":
                return "torch"
            if not native.kernels_available():
                # never a silent downgrade on a GPU: the kernel library is part of the build
                raise RuntimeError(f"{native.KERNELS_SO} is missing on a GPU device: build it "
                                   "(__graft_entry__.build()) or pass backend='torch'")
            try:
                fused.supports(self, explain=True)
                return "fused"
            except RuntimeError as e:
                logging.getLogger("gfedntm_amd").warning(
                    "%s; this configuration runs on the PyTorch engine", e)
                # recorded (engine_info: bench / metrics records say which engine ran)
                self.backend_fallback_reason = str(e)
                return "torch"
        if backend == "fused":
            from ..ops import engine as fused
            if not fused.supports(self, explain=True):
                raise RuntimeError("fused backend does not support this configuration")
        return backend

    FUSED_SHARED_LAST = ("inf_net.adapt_bert.weight", "inf_net.adapt_bert.bias", "beta")

    def _build_engine(self):
        transposed = TRANSPOSED_KEYS if self.backend == "fused" else ()
        padded = {}
        if self.backend == "fused":
            from ..ops.engine import BETA_PAD, BETA_PAD_MIN_V
            if self.input_size >= BETA_PAD_MIN_V:
                padded = {"beta": BETA_PAD}        # beta rows of whole 64-column tiles (utils/flat.py)
        self.flat = FlatState(self.model, self.shared_keys, transposed=transposed,
                              device=self.device,
                              # (the shared tail in the order its parts become final in
                              # a fused step: CombinedTM's adapt_bert after ctx_bwd, beta
                              # after the decoder backward -- ops/engine.py attach_fedavg)
                              shared_last=self.FUSED_SHARED_LAST if self.backend == "fused" else (),
                              padded=padded)
        if self.backend == "fused":
            from ..ops.engine import FusedEngine
            self.engine = FusedEngine(self)
        else:
            self.engine = TorchEngine(self.model, self.flat, self.solver, self.lr,
                                      self.momentum, self.reduce_on_plateau,
                                      float(self.weights.get("beta", 1)), kind=self.kind)
        self.optimizer = self.engine.optimizer
        self.USE_CUDA = self.device.type == "cuda"

    # ---------------------------------------------------------------- data
    def device_data(self, dataset) -> DeviceCSR:
        key = id(dataset)
        if key not in self._device_data:
            ctx = getattr(dataset, "X_contextual", None)
            lab = getattr(dataset, "labels", None)
            self._device_data[key] = DeviceCSR(dataset.csr, self.device, ctx, lab)
        return self._device_data[key]

    # ---------------------------------------------------------------- loss
    def _loss(self, inputs, word_dists, prior_mean, prior_variance, posterior_mean,
              posterior_variance, posterior_log_variance):
        """Sum over the batch of KL + RL (reference avitm.py:168-229)."""
        kl = kl_terms(prior_mean, prior_variance, posterior_mean, posterior_variance,
                      posterior_log_variance, self.n_components)
        rl = reconstruction_terms(inputs, word_dists)
        return (kl + rl).sum()

    # ---------------------------------------------------------------- training
    def _run_plan(self, data: DeviceCSR, plan: BatchPlan):
        self.engine.bind_data(data, plan)
        self.model.train()
        for s in range(plan.n_steps):
            self.engine.step(s)
        return float(self.engine.loss_hist.sum().item())

    def _train_epoch(self, loader_or_dataset, seed: int = 0):
        """One epoch over a dataset; returns (samples_processed, mean train loss)."""
        ds = loader_or_dataset.dataset if hasattr(loader_or_dataset, "dataset") else \
            loader_or_dataset
        data = self.device_data(ds)
        plan = BatchPlan.build(data.n_docs, self.batch_size,
                               -(-data.n_docs // self.batch_size), seed=seed)
        total = self._run_plan(data, plan)
        return data.n_docs, total / data.n_docs

    @torch.no_grad()
    def _validate_epoch(self, loader_or_dataset):
        ds = loader_or_dataset.dataset if hasattr(loader_or_dataset, "dataset") else \
            loader_or_dataset
        data = self.device_data(ds)
        was = self.model.training
        self.model.eval()
        total = 0.0
        for a in range(0, data.n_docs, self.batch_size):
            ids = torch.arange(a, min(a + self.batch_size, data.n_docs), device=self.device)
            total += float(self._batch_loss(data, ids).item())
        self.model.train(was)
        return data.n_docs, total / max(data.n_docs, 1)

    def _batch_loss(self, data: DeviceCSR, ids):
        raise NotImplementedError

    def fit(self, train_dataset, validation_dataset=None, save_dir=None, patience=5, delta=0,
            n_samples=20):
        if self.verbose:
            self.logger.info(
                "Settings: N Components: %s Topic Prior Mean: %s Topic Prior Variance: %s "
                "Model Type: %s Hidden Sizes: %s Activation: %s Dropout: %s Learn Priors: %s "
                "Learning Rate: %s Momentum: %s Reduce On Plateau: %s Save Dir: %s",
                self.n_components, self.topic_prior_mean, self.topic_prior_variance,
                self.model_type, self.hidden_sizes, self.activation, self.dropout,
                self.learn_priors, self.lr, self.momentum, self.reduce_on_plateau, save_dir)
        self.model_dir = save_dir
        self.train_data = train_dataset
        self.validation_data = validation_dataset
        if validation_dataset is not None:
            self.early_stopping = EarlyStopping(patience=patience, verbose=self.verbose,
                                                path=save_dir, delta=delta)
        samples_processed = 0
        for epoch in range(self.num_epochs):
            self.nn_epoch = epoch
            s = datetime.datetime.now()
            sp, train_loss = self._train_epoch(train_dataset, seed=epoch)
            samples_processed += sp
            e = datetime.datetime.now()
            self.best_components = self.model.beta
            if validation_dataset is not None:
                vsp, val_loss = self._validate_epoch(validation_dataset)
                if self.verbose:
                    self.logger.info("Epoch: [%d/%d]\tSamples: [%d/%d]\tValidation Loss: %s\tTime: %s",
                                     epoch + 1, self.num_epochs, vsp,
                                     len(validation_dataset) * self.num_epochs, val_loss, e - s)
                if np.isnan(val_loss) or np.isnan(train_loss):
                    break
                self.early_stopping(val_loss, self)
                if self.early_stopping.early_stop:
                    self.logger.info("Early stopping")
                    break
            elif save_dir is not None:
                self.save(save_dir)
            if self.verbose:
                self.logger.info("Epoch: [%d/%d]\t Seen Samples: [%d/%d]\tTrain Loss: %s\tTime: %s",
                                 epoch + 1, self.num_epochs, samples_processed,
                                 len(train_dataset) * self.num_epochs, train_loss, e - s)
        self.training_doc_topic_distributions = self.get_doc_topic_distribution(
            train_dataset, n_samples)

    # ---------------------------------------------------------------- inference
    @torch.no_grad()
    def _posterior(self, data: DeviceCSR, ids):
        raise NotImplementedError

    @torch.no_grad()
    def get_doc_topic_distribution(self, dataset, n_samples=20, seed: Optional[int] = None,
                                   chunk: int = 4096):
        """Mean over ``n_samples`` reparameterised draws of softmax(theta), per doc.
        Fused engine: one HIP launch per chunk (csrc/infer.hip), encoder evaluated once
        per document; torch engine: encoder once per chunk, draws from torch."""
        data = self.device_data(dataset)
        if seed is None:
            seed = int(torch.initial_seed()) % (2**31)
        if self.backend == "fused":
            return self.engine.theta_infer(data, n_samples, seed=seed).cpu().numpy()
        was = self.model.training
        self.model.eval()
        gen = torch.Generator(device=self.device)
        gen.manual_seed(seed)
        out = []
        for a in range(0, data.n_docs, chunk):
            ids = torch.arange(a, min(a + chunk, data.n_docs), device=self.device)
            mu, logvar = self._posterior(data, ids)
            out.append(sample_theta_mean(mu, logvar, n_samples, gen))
        self.model.train(was)
        if not out:
            return np.zeros((0, self.n_components), dtype=np.float32)
        return torch.cat(out).cpu().numpy()

    def get_predicted_topics(self, dataset, n_samples):
        thetas = self.get_doc_topic_distribution(dataset, n_samples)
        return [int(np.argmax(t / np.sum(t))) for t in thetas]

    @torch.no_grad()
    def topic_word_matrix_tensor(self) -> torch.Tensor:
        """ProdLDA: beta.  NeuralLDA: softmax_V(BN_K(beta)) with batch statistics,
        i.e. what the last training forward stored (reference decoder_network.py:121-132)."""
        beta = self.model.beta.detach()
        if self.model.is_prodlda:
            return beta
        mean = beta.mean(0, keepdim=True)
        var = beta.var(0, unbiased=False, keepdim=True)
        bn = (beta - mean) / torch.sqrt(var + self.model.beta_batchnorm.eps)
        return torch.softmax(bn, dim=1)

    def get_topic_word_matrix(self):
        return self.topic_word_matrix_tensor().cpu().numpy()

    def get_topic_word_distribution(self):
        """softmax over V of the topic-word matrix (reference avitm.py:539-551).  For
        NeuralLDA the reference softmaxes an already-normalised matrix (B9); that is kept
        when ``compat_double_softmax`` is True."""
        m = self.topic_word_matrix_tensor()
        if not self.model.is_prodlda and not self.compat_double_softmax:
            return m.cpu().numpy()
        return torch.softmax(m.double(), dim=1).cpu().numpy()

    def get_topics(self, k=10):
        if k > self.input_size:
            raise ValueError("k must be <= input size")
        comps = self.best_components if self.best_components is not None else self.model.beta
        idx2token = self._idx2token()
        _, idxs = torch.topk(comps.detach(), k, dim=1)
        return [[idx2token[int(i)] for i in row] for row in idxs.cpu().numpy()]

    def _idx2token(self):
        td = self.train_data
        if td is not None and getattr(td, "idx2token", None) is not None:
            return td.idx2token
        return {i: str(i) for i in range(self.input_size)}

    # ---------------------------------------------------------------- persistence
    def _format_file(self):
        pv = (self.topic_prior_variance if self.topic_prior_variance is not None
              else 1 - 1.0 / self.n_components)
        return "{}_nc_{}_tpm_{}_tpv_{}_hs_{}_ac_{}_do_{}_lr_{}_mo_{}_rp_{}".format(
            self.model_dir_prefix, self.n_components, self.topic_prior_mean, pv,
            self.hidden_sizes, self.activation, self.dropout, self.lr, self.momentum,
            self.reduce_on_plateau)

    def config_dict(self) -> Dict[str, Any]:
        keys = ["input_size", "n_components", "model_type", "hidden_sizes", "activation",
                "dropout", "learn_priors", "batch_size", "lr", "momentum", "solver",
                "num_epochs", "reduce_on_plateau", "topic_prior_mean", "topic_prior_variance",
                "num_samples", "nn_epoch", "best_loss_train",
                "matmul_dtype"]
        return {k: getattr(self, k) for k in keys}

    def save(self, models_dir=None):
        if self.model is None or models_dir is None:
            return
        d = os.path.join(models_dir, self._format_file())
        os.makedirs(d, exist_ok=True)
        path = os.path.join(d, f"epoch_{self.nn_epoch}.pth")
        torch.save({"state_dict": self.model.state_dict(),
                    "optimizer": self.engine.optimizer_state_dict(),
                    "dcue_dict": self.config_dict()}, path)
        return path

    def load(self, model_dir, epoch):
        path = os.path.join(model_dir, f"epoch_{epoch}.pth")
        ck = torch.load(path, map_location=self.device, weights_only=True)
        for k, v in ck.get("dcue_dict", {}).items():
            if k in ("nn_epoch", "best_loss_train"):
                setattr(self, k, v)
        self.model.load_state_dict(ck["state_dict"])
        if "optimizer" in ck and ck["optimizer"] is not None:
            self.engine.load_optimizer_state_dict(ck["optimizer"])


def sample_theta_mean(mu: torch.Tensor, logvar: torch.Tensor, n_samples: int,
                      gen: torch.Generator) -> torch.Tensor:
    """mean_s softmax(mu + eps_s * exp(logvar / 2)) with the encoder evaluated once."""
    std = torch.exp(0.5 * logvar)
    acc = torch.zeros_like(mu)
    for _ in range(n_samples):
        eps = torch.randn(mu.shape, generator=gen, device=mu.device, dtype=mu.dtype)
        acc += F.softmax(mu + eps * std, dim=1)
    return acc / n_samples
