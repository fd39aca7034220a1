"""Pure-PyTorch neural topic model networks (the numerical oracle).

These modules define the exact math of the reference models and keep their
``state_dict`` key names and parameter order byte-for-byte compatible, because
keys are the wire/checkpoint contract (reference ModelUpdate fields,
src/protos/federated.proto:144-170, and the 22-key ``grads_to_share`` list).

Reference parity:
  * AVITM encoder      -- src/models/base/pytorchavitm/avitm_network/inference_network.py:7-85
  * AVITM decoder      -- .../avitm_network/decoder_network.py:10-147
  * CTM encoders       -- src/models/base/contextualized_topic_models/ctm_network/inference_network.py:6-193
  * CTM decoder        -- .../ctm_network/decoding_network.py:8-174

The MI355X training path does not run these modules: it runs the fused HIP
engine in :mod:`gfedntm_amd.ops.engine`, whose flat parameter buffer is
exposed back through a module of this file (parameters become views into the
flat buffer), so checkpoints and the wire format stay identical.

Fixed reference defects: B12 (``if labels:`` on a
tensor in the zero-shot encoder) is fixed here.
"""
from __future__ import annotations

from collections import OrderedDict
from typing import Optional, Sequence, Tuple

import torch
from torch import nn
from torch.nn import functional as F

ACTIVATIONS = ("softplus", "relu", "sigmoid", "tanh", "leakyrelu", "rrelu", "elu", "selu")


def make_activation(name: str) -> nn.Module:
    table = {
        "softplus": nn.Softplus, "relu": nn.ReLU, "sigmoid": nn.Sigmoid,
        "tanh": nn.Tanh, "leakyrelu": nn.LeakyReLU, "rrelu": nn.RReLU,
        "elu": nn.ELU, "selu": nn.SELU,
    }
    if name not in table:
        raise ValueError(f"activation must be one of {ACTIVATIONS}, got {name!r}")
    return table[name]()


def _check_hidden(hidden_sizes):
    if not isinstance(hidden_sizes, tuple) or len(hidden_sizes) < 1:
        raise TypeError("hidden_sizes must be a non-empty tuple")


class _EncoderTrunk(nn.Module):
    """Hidden MLP + dropout + (mu, log sigma^2) heads with BN(affine=False).

    Subclasses create ``input_layer`` (and ``adapt_bert`` for the combined
    encoder) *before* calling :meth:`_build_trunk` so that parameter
    registration order matches the reference (Adam param ids depend on it).
    """

    def _build_trunk(self, hidden_sizes, output_size, activation, dropout):
        pairs = list(zip(hidden_sizes[:-1], hidden_sizes[1:]))
        self.hiddens = nn.Sequential(OrderedDict(
            (f"l_{i}", nn.Sequential(nn.Linear(a, b), self.activation))
            for i, (a, b) in enumerate(pairs)))
        self.f_mu = nn.Linear(hidden_sizes[-1], output_size)
        self.f_mu_batchnorm = nn.BatchNorm1d(output_size, affine=False)
        self.f_sigma = nn.Linear(hidden_sizes[-1], output_size)
        self.f_sigma_batchnorm = nn.BatchNorm1d(output_size, affine=False)
        self.dropout_enc = nn.Dropout(p=dropout)

    def _trunk(self, h0_pre: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        h = self.activation(h0_pre)
        h = self.hiddens(h)
        h = self.dropout_enc(h)
        mu = self.f_mu_batchnorm(self.f_mu(h))
        log_sigma = self.f_sigma_batchnorm(self.f_sigma(h))
        return mu, log_sigma


class InferenceNetwork(_EncoderTrunk):
    """AVITM bag-of-words encoder: x[B,V] -> (mu, log sigma^2)[B,K]."""

    def __init__(self, input_size: int, output_size: int, hidden_sizes: Sequence[int],
                 activation: str = "softplus", dropout: float = 0.2):
        super().__init__()
        _check_hidden(hidden_sizes)
        if dropout < 0:
            raise ValueError("dropout must be >= 0")
        self.input_size, self.output_size = input_size, output_size
        self.hidden_sizes, self.dropout = hidden_sizes, dropout
        self.activation = make_activation(activation)
        self.input_layer = nn.Linear(input_size, hidden_sizes[0])
        self._build_trunk(hidden_sizes, output_size, activation, dropout)

    def forward(self, x: torch.Tensor):
        return self._trunk(self.input_layer(x))


class CombinedInferenceNetwork(_EncoderTrunk):
    """CombinedTM encoder: concat(BoW, adapt_bert(x_bert)[, labels]) -> MLP."""

    def __init__(self, input_size: int, bert_size: int, output_size: int,
                 hidden_sizes: Sequence[int], activation: str = "softplus",
                 dropout: float = 0.2, label_size: int = 0):
        super().__init__()
        _check_hidden(hidden_sizes)
        self.input_size, self.output_size = input_size, output_size
        self.hidden_sizes, self.dropout = hidden_sizes, dropout
        self.activation = make_activation(activation)
        self.adapt_bert = nn.Linear(bert_size, input_size)
        self.input_layer = nn.Linear(2 * input_size + label_size, hidden_sizes[0])
        self._build_trunk(hidden_sizes, output_size, activation, dropout)

    def forward(self, x, x_bert, labels: Optional[torch.Tensor] = None):
        parts = [x, self.adapt_bert(x_bert)]
        if labels is not None:
            parts.append(labels)
        return self._trunk(self.input_layer(torch.cat(parts, dim=1)))


class ContextualInferenceNetwork(_EncoderTrunk):
    """ZeroShotTM encoder: only the contextual embedding (+labels) is encoded."""

    def __init__(self, input_size: int, bert_size: int, output_size: int,
                 hidden_sizes: Sequence[int], activation: str = "softplus",
                 dropout: float = 0.2, label_size: int = 0):
        super().__init__()
        _check_hidden(hidden_sizes)
        self.input_size, self.output_size = input_size, output_size
        self.hidden_sizes, self.dropout = hidden_sizes, dropout
        self.activation = make_activation(activation)
        self.input_layer = nn.Linear(bert_size + label_size, hidden_sizes[0])
        self._build_trunk(hidden_sizes, output_size, activation, dropout)

    def forward(self, x, x_bert, labels: Optional[torch.Tensor] = None):
        # reference used `if labels:` on a tensor (B12); test for None instead
        h = x_bert if labels is None else torch.cat((x_bert, labels), 1)
        return self._trunk(self.input_layer(h))


class _TopicDecoder(nn.Module):
    """Shared prior + theta sampling + ProdLDA/LDA word-distribution decoder."""

    def _build_decoder(self, input_size, n_components, model_type, dropout, learn_priors,
                       topic_prior_mean, topic_prior_variance):
        if model_type.lower() not in ("prodlda", "lda"):
            raise ValueError("model type must be 'prodLDA' or 'LDA'")
        self.input_size, self.n_components = input_size, n_components
        self.model_type, self.dropout, self.learn_priors = model_type, dropout, learn_priors
        pm = torch.full((n_components,), float(topic_prior_mean))
        if topic_prior_variance is None:
            topic_prior_variance = 1.0 - 1.0 / n_components
        pv = torch.full((n_components,), float(topic_prior_variance))
        if learn_priors:
            self.prior_mean = nn.Parameter(pm)
            self.prior_variance = nn.Parameter(pv)
        else:
            self.register_buffer("prior_mean", pm, persistent=False)
            self.register_buffer("prior_variance", pv, persistent=False)
        self.beta = nn.Parameter(torch.empty(n_components, input_size))
        nn.init.xavier_uniform_(self.beta)

    def _build_tail(self, input_size):
        self.beta_batchnorm = nn.BatchNorm1d(input_size, affine=False)
        self.drop_theta = nn.Dropout(p=self.dropout)

    @property
    def is_prodlda(self) -> bool:
        return self.model_type.lower() == "prodlda"

    @staticmethod
    def reparameterize(mu, logvar):
        return torch.randn_like(mu) * torch.exp(0.5 * logvar) + mu

    def _decode(self, mu, log_sigma):
        theta = F.softmax(self.reparameterize(mu, log_sigma), dim=1)
        theta = self.drop_theta(theta)
        if self.is_prodlda:
            word_dist = F.softmax(self.beta_batchnorm(theta @ self.beta), dim=1)
            twm = self.beta
        else:
            beta = F.softmax(self.beta_batchnorm(self.beta), dim=1)
            word_dist = theta @ beta
            twm = beta
        # plain attribute: the reference's assignment registered beta a second time
        # as a parameter named topic_word_matrix; keep the state_dict free of that alias
        object.__setattr__(self, "topic_word_matrix", twm)
        return theta, word_dist


class DecoderNetwork(_TopicDecoder):
    """AVITM (ProdLDA / NeuralLDA) VAE.  forward(x) -> 6-tuple like the reference."""

    def __init__(self, input_size: int, n_components: int = 10, model_type: str = "prodLDA",
                 hidden_sizes=(100, 100), activation: str = "softplus", dropout: float = 0.2,
                 learn_priors: bool = True, topic_prior_mean: float = 0.0,
                 topic_prior_variance: Optional[float] = None):
        super().__init__()
        self.hidden_sizes, self.activation = hidden_sizes, activation
        self.inf_net = InferenceNetwork(input_size, n_components, hidden_sizes, activation)
        self._build_decoder(input_size, n_components, model_type, dropout, learn_priors,
                            topic_prior_mean, topic_prior_variance)
        self._build_tail(input_size)
        object.__setattr__(self, "topic_word_matrix", None)

    def forward(self, x):
        mu, log_sigma = self.inf_net(x)
        _, word_dist = self._decode(mu, log_sigma)
        return (self.prior_mean, self.prior_variance, mu, torch.exp(log_sigma),
                log_sigma, word_dist)

    @torch.no_grad()
    def get_theta(self, x):
        mu, log_sigma = self.inf_net(x)
        return F.softmax(self.reparameterize(mu, log_sigma), dim=1)


class CTMDecoderNetwork(_TopicDecoder):
    """CTM VAE (combined or zero-shot encoder).  forward -> 7-tuple like the reference."""

    def __init__(self, input_size: int, contextual_size: int, infnet: str = "combined",
                 n_components: int = 10, model_type: str = "prodLDA", hidden_sizes=(100, 100),
                 activation: str = "softplus", dropout: float = 0.2, learn_priors: bool = True,
                 topic_prior_mean: float = 0.0, topic_prior_variance: Optional[float] = None,
                 label_size: int = 0):
        super().__init__()
        if model_type not in ("prodLDA", "LDA"):
            raise ValueError("model type must be 'prodLDA' or 'LDA'")
        self.hidden_sizes, self.activation, self.infnet = hidden_sizes, activation, infnet
        self.label_size = label_size
        if infnet == "zeroshot":
            self.inf_net = ContextualInferenceNetwork(
                input_size, contextual_size, n_components, hidden_sizes, activation,
                label_size=label_size)
        elif infnet == "combined":
            self.inf_net = CombinedInferenceNetwork(
                input_size, contextual_size, n_components, hidden_sizes, activation,
                label_size=label_size)
        else:
            raise ValueError("infnet must be 'zeroshot' or 'combined'")
        if label_size:
            self.label_classification = nn.Linear(n_components, label_size)
        self._build_decoder(input_size, n_components, model_type, dropout, learn_priors,
                            topic_prior_mean, topic_prior_variance)
        self._build_tail(input_size)
        object.__setattr__(self, "topic_word_matrix", None)

    def forward(self, x, x_bert, labels=None):
        mu, log_sigma = self.inf_net(x, x_bert, labels)
        theta, word_dist = self._decode(mu, log_sigma)
        est = self.label_classification(theta) if labels is not None else None
        return (self.prior_mean, self.prior_variance, mu, torch.exp(log_sigma), log_sigma,
                word_dist, est)

    @torch.no_grad()
    def get_theta(self, x, x_bert, labels=None):
        mu, log_sigma = self.inf_net(x, x_bert, labels)
        return F.softmax(self.reparameterize(mu, log_sigma), dim=1)


def kl_terms(prior_mean, prior_variance, post_mean, post_var, post_logvar, n_components):
    """Per-document KL(q || p) of two diagonal Gaussians (reference avitm.py:207-220)."""
    var_division = torch.sum(post_var / prior_variance, dim=1)
    diff = prior_mean - post_mean
    diff_term = torch.sum(diff * diff / prior_variance, dim=1)
    logdet = prior_variance.log().sum() - post_logvar.sum(dim=1)
    return 0.5 * (var_division + diff_term - n_components + logdet)


def reconstruction_terms(x, word_dists):
    """Per-document multinomial NLL with the reference's +1e-10 (avitm.py:225)."""
    return -torch.sum(x * torch.log(word_dists + 1e-10), dim=1)
