"""Contextualized topic models: CombinedTM and ZeroShotTM
(reference src/models/base/contextualized_topic_models/ctm_network/ctm.py:20-807)."""
from __future__ import annotations

import numpy as np
import torch

from ..data.bow import DeviceCSR
from .networks import CTMDecoderNetwork
from .topic_model import TopicModelBase


class CTM(TopicModelBase):
    kind = "ctm"
    model_dir_prefix = "contextualized_topic_model"

    def __init__(self, logger=None, input_size: int = 0, contextual_size: int = 768,
                 inference_type: str = "combined", label_size: int = 0, **kw):
        self.contextual_size = int(contextual_size)
        self.inference_type = inference_type
        self.label_size = int(label_size)
        if kw.get("model_type", "prodLDA") not in ("prodLDA", "LDA"):
            raise ValueError("model must be 'LDA' or 'prodLDA'")
        super().__init__(logger=logger, input_size=input_size, **kw)

    def _build_network(self, **extra):
        return CTMDecoderNetwork(self.input_size, self.contextual_size, self.inference_type,
                                 self.n_components, self.model_type, self.hidden_sizes,
                                 self.activation, self.dropout, self.learn_priors,
                                 self.topic_prior_mean, self.topic_prior_variance,
                                 label_size=self.label_size)

    def _inputs(self, data: DeviceCSR, ids):
        x = data.dense_rows(ids)
        ctx = data.contextual[ids]
        lab = data.labels[ids] if data.labels is not None else None
        return x, ctx, lab

    def _loss(self, inputs, word_dists, prior_mean, prior_variance, posterior_mean,
              posterior_variance, posterior_log_variance):
        """Returns (KL, RL) per document, like the reference CTM._loss (ctm.py:182-238)."""
        from .networks import kl_terms, reconstruction_terms
        kl = kl_terms(prior_mean, prior_variance, posterior_mean, posterior_variance,
                      posterior_log_variance, self.n_components)
        return kl, reconstruction_terms(inputs, word_dists)

    def _batch_loss(self, data: DeviceCSR, ids):
        x, ctx, lab = self._inputs(data, ids)
        pm, pv, mu, var, logvar, wd, est = self.model(x, ctx, lab)
        kl, rl = self._loss(x, wd, pm, pv, mu, var, logvar)
        loss = (self.weights["beta"] * kl + rl).sum()
        if lab is not None:
            loss = loss + torch.nn.functional.cross_entropy(est, torch.argmax(lab, 1))
        return loss

    @torch.no_grad()
    def _posterior(self, data: DeviceCSR, ids):
        x, ctx, lab = self._inputs(data, ids)
        return self.model.inf_net(x, ctx, lab)

    def config_dict(self):
        d = super().config_dict()
        d.update(contextual_size=self.contextual_size, inference_type=self.inference_type,
                 label_size=self.label_size)
        return d

    # ------------------------------------------------------------- CTM extras
    def get_word_distribution_by_topic_id(self, topic):
        if topic >= self.n_components:
            raise ValueError("Topic id must be lower than the number of topics")
        wd = self.get_topic_word_distribution()
        t = [(word, wd[topic][idx]) for idx, word in self._idx2token().items()]
        return sorted(t, key=lambda x: -x[1])

    def get_top_documents_per_topic_id(self, unpreprocessed_corpus, document_topic_distributions,
                                       topic_id, k=5):
        probs = document_topic_distributions.T[topic_id]
        ind = probs.argsort()[-k:][::-1]
        return [(unpreprocessed_corpus[i], document_topic_distributions[i][topic_id]) for i in ind]

    def get_most_likely_topic(self, doc_topic_distribution):
        return np.argmax(doc_topic_distribution, axis=0)

    def get_ldavis_data_format(self, vocab, dataset, n_samples):
        term_frequency = np.ravel(dataset.X_bow.sum(axis=0))
        doc_lengths = np.ravel(dataset.X_bow.sum(axis=1))
        return {"topic_term_dists": self.get_topic_word_distribution(),
                "doc_topic_dists": self.get_doc_topic_distribution(dataset, n_samples=n_samples),
                "doc_lengths": doc_lengths, "vocab": vocab, "term_frequency": term_frequency}


class ZeroShotTM(CTM):
    """ZeroShotTM (Bianchi et al., EACL 2021): contextual-only encoder."""

    def __init__(self, **kwargs):
        super().__init__(**kwargs, inference_type="zeroshot")


class CombinedTM(CTM):
    """CombinedTM (Bianchi et al., ACL 2021): BoW + adapted contextual encoder."""

    def __init__(self, **kwargs):
        super().__init__(**kwargs, inference_type="combined")
