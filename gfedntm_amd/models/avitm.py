"""AVITM trainer: ProdLDA and NeuralLDA on bag-of-words
(reference src/models/base/pytorchavitm/avitm_network/avitm.py:20-640)."""
from __future__ import annotations

import torch

from ..data.bow import DeviceCSR
from .networks import DecoderNetwork
from .topic_model import TopicModelBase


class AVITM(TopicModelBase):
    kind = "avitm"
    model_dir_prefix = "AVITM"

    def _build_network(self, **extra):
        return DecoderNetwork(self.input_size, self.n_components, self.model_type,
                              self.hidden_sizes, self.activation, self.dropout,
                              self.learn_priors, self.topic_prior_mean,
                              self.topic_prior_variance)

    def _batch_loss(self, data: DeviceCSR, ids):
        x = data.dense_rows(ids)
        pm, pv, mu, var, logvar, wd = self.model(x)
        return self._loss(x, wd, pm, pv, mu, var, logvar)

    @torch.no_grad()
    def _posterior(self, data: DeviceCSR, ids):
        return self.model.inf_net(data.dense_rows(ids))
