"""Functional forward of the topic VAEs with *explicit* noise.

The module forward (networks.py) draws its own dropout masks and Gaussian
noise; the fused kernels draw theirs from a Philox stream.  To compare the two
bit-for-bit up to float rounding, this file re-states the training forward
(reference decoder_network.py:109-135, inference_network.py:76-85) with the
noise passed in: ``eps`` [B,K], ``mask_h`` [B,H_last] and ``mask_t`` [B,K]
(inverted-dropout scales: 0 or 1/(1-p)).  It is the oracle of
tests/test_fused_kernels.py and uses the module's own parameters, so autograd
gives the reference gradients.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .networks import kl_terms, reconstruction_terms


def encoder_forward(net, x_in: torch.Tensor, mask_h: torch.Tensor, bn_training: bool = True):
    h = net.activation(net.input_layer(x_in))
    h = net.hiddens(h)
    h = h * mask_h
    bn = net.f_mu_batchnorm
    mu = F.batch_norm(net.f_mu(h), bn.running_mean, bn.running_var, training=bn_training,
                      momentum=bn.momentum, eps=bn.eps)
    bs = net.f_sigma_batchnorm
    ls = F.batch_norm(net.f_sigma(h), bs.running_mean, bs.running_var, training=bn_training,
                      momentum=bs.momentum, eps=bs.eps)
    if bn_training:
        bn.num_batches_tracked += 1
        bs.num_batches_tracked += 1
    return mu, ls


def decoder_forward(model, mu, ls, eps, mask_t):
    theta = F.softmax(mu + eps * torch.exp(0.5 * ls), dim=1)
    thetad = theta * mask_t
    bb = model.beta_batchnorm
    if model.is_prodlda:
        logits = F.batch_norm(thetad @ model.beta, bb.running_mean, bb.running_var,
                              training=True, momentum=bb.momentum, eps=bb.eps)
        word_dist = F.softmax(logits, dim=1)
    else:
        bnb = F.batch_norm(model.beta, bb.running_mean, bb.running_var, training=True,
                           momentum=bb.momentum, eps=bb.eps)
        word_dist = thetad @ F.softmax(bnb, dim=1)
    bb.num_batches_tracked += 1
    return theta, thetad, word_dist


def avitm_loss_explicit(model, x, eps, mask_h, mask_t, kl_weight: float = 1.0, x_enc=None):
    """Sum over the batch of kl_weight*KL + RL with explicit noise.

    ``x_enc`` is the encoder input when it differs from the BoW (CTM)."""
    mu, ls = encoder_forward(model.inf_net, x if x_enc is None else x_enc, mask_h)
    _, _, wd = decoder_forward(model, mu, ls, eps, mask_t)
    kl = kl_terms(model.prior_mean, model.prior_variance, mu, torch.exp(ls), ls,
                  model.n_components)
    rl = reconstruction_terms(x, wd)
    return (kl_weight * kl + rl).sum(), kl, rl
