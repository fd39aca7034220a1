"""Split W_in update (csrc/update.hip gfk_win_dense_k + win_tile_sparse_rows).

At large vocabularies the input layer's Adam step is split: the words of the batch are
updated by the sparse tiles after the encoder backward, every other word (zero gradient)
by a streaming kernel forked onto a side stream after post_fwd.  The two halves must
reproduce the one-kernel update bit for bit -- parameters, both Adam moments and the
losses -- with the FedAvg pre-scale, across epochs (word stamps are generations, never
step indices), in graph replays, and in batched multi-client launches.
"""
import pytest
import torch

from gfedntm_amd.data.bow import BatchPlan, DeviceCSR
from gfedntm_amd.models import AVITM
from gfedntm_amd.ops import kernel_abi as abi
from gfedntm_amd.ops.engine import (STAGE_WIN_SPARSE, STAGE_WIN_SPLIT, STAGE_WIN_VREG, UPDATE_FUSED,
                                     UPDATE_GRAD)
from tests.helpers import random_csr

pytestmark = pytest.mark.gpu


def _make(monkeypatch, split, model_type, V, K, H, B=64, seed=0):
    monkeypatch.setenv("GFEDNTM_WIN_SPARSE", "1")
    monkeypatch.setenv("GFEDNTM_WIN_SPLIT", split)
    torch.manual_seed(seed)
    return AVITM(input_size=V, n_components=K, model_type=model_type, hidden_sizes=H,
                 batch_size=B, verbose=False, device="cuda", backend="fused")


def _run(tm, X, n_steps, B, graph, scale=0.75):
    data = DeviceCSR(X, "cuda")
    plan = BatchPlan.build(data.n_docs, B, n_steps, seed=3)
    tm.engine.set_fedavg_scale(scale)
    tm.engine.bind_data(data, plan)
    tm.engine.enable_graph(graph)
    for s in range(n_steps):
        tm.engine.step(s)
    torch.cuda.synchronize()


def _assert_same_state(a, b):
    ea, eb = a.engine, b.engine
    assert torch.equal(ea.loss_hist, eb.loss_hist)
    for name in ("buffer",):
        assert torch.equal(getattr(ea.flat, name), getattr(eb.flat, name))
    assert torch.equal(ea.exp_avg, eb.exp_avg)
    assert torch.equal(ea.exp_avg_sq, eb.exp_avg_sq)


@pytest.mark.parametrize("model_type", ["prodLDA", "LDA"])
@pytest.mark.parametrize("V,K,H,B,n_docs,graph", [
    (20000, 20, (50, 50), 64, 150, True),      # 3 epochs of 3 batches (stamps across epochs)
    (30000, 50, (64,), 32, 90, False),         # H0 = 64, eager launches
    (9000, 30, (30, 20), 128, 300, True),      # H0 = 30 (quads span two words), B = 128
])
def test_split_win_update_is_bit_identical(monkeypatch, model_type, V, K, H, B, n_docs, graph):
    a = _make(monkeypatch, "0", model_type, V, K, H, B)
    b = _make(monkeypatch, "1", model_type, V, K, H, B)
    b.model.load_state_dict(a.model.state_dict())
    b.engine.seed = b.engine._m.seed = a.engine.seed
    assert a.engine._m.stage_flags & STAGE_WIN_SPARSE and not a.engine.win_split
    assert b.engine.win_split and abi.PH_WIN_FORK in b.engine.phases()
    X = random_csr(n_docs, V, 60, seed=5)
    n_steps = 3 * -(-n_docs // B)
    for tm in (a, b):
        _run(tm, X, n_steps, B, graph)
    _assert_same_state(a, b)


def test_split_follows_update_mode(monkeypatch):
    """Gradient mode turns the split off (the generic optimizer owns W_in); switching back
    re-prepares the bound batch's word stamps, so the next fused steps stay exact."""
    V, K, H, B = 20000, 20, (50, 50), 64
    a = _make(monkeypatch, "0", "prodLDA", V, K, H, B)
    b = _make(monkeypatch, "1", "prodLDA", V, K, H, B)
    b.model.load_state_dict(a.model.state_dict())
    b.engine.seed = b.engine._m.seed = a.engine.seed
    X = random_csr(150, V, 60, seed=6)
    for tm in (a, b):
        data = DeviceCSR(X, "cuda")
        tm.engine.bind_data(data, BatchPlan.build(data.n_docs, B, 6, seed=1))
        tm.engine.set_update_mode(UPDATE_GRAD)
        assert not tm.engine.win_split
        tm.engine.step(0)
        tm.engine.step(1)
        tm.engine.set_update_mode(UPDATE_FUSED)
        for s in range(2, 6):
            tm.engine.step(s)
    torch.cuda.synchronize()
    assert b.engine.win_split
    _assert_same_state(a, b)


def test_split_batched_clients_match_unsplit(monkeypatch):
    """LocalFederation's batched launches (grid z = client) fork the dense half once for
    all clients: the rounds equal the unsplit batched rounds bit for bit."""
    from gfedntm_amd.data.synthetic import generate_synthetic
    from gfedntm_amd.federation.data import ClientCorpus
    from gfedntm_amd.federation.runner import LocalFederation
    from gfedntm_amd.utils.config import load_config
    monkeypatch.setenv("GFEDNTM_WIN_SPARSE", "1")
    sc = generate_synthetic(vocab_size=12000, n_topics=10, n_docs=90, n_nodes=3, frozen_topics=2,
                            nwords=(60, 120), seed=12)
    corpora = [ClientCorpus(synthetic=sc, node=i) for i in range(3)]
    p = dict(load_config().training_params)
    p.update(num_epochs=2, batch_size=32, hidden_sizes=(50, 50), n_components=10)
    outs = []
    for split in ("0", "1"):
        monkeypatch.setenv("GFEDNTM_WIN_SPLIT", split)
        fed = LocalFederation(corpora, p, max_iters=8, round_batched=True, device="cuda",
                              backend="fused", seed=4)
        fed.run()
        torch.cuda.synchronize()
        assert fed._batched is not None
        assert fed.clients[0].tm.engine.win_split == (split == "1")
        outs.append([c.tm.flat.buffer.clone() for c in fed.clients])
    for x, y in zip(*outs):
        assert torch.equal(x, y)


@pytest.mark.parametrize("V,K,H,B,n_docs,graph", [
    (20000, 20, (50, 50), 64, 150, True),
    (9000, 30, (30, 20), 128, 300, False),     # quads spanning two words
    (300, 20, (32,), 128, 300, True),          # > 512 entries per tile: several list passes
])
def test_lds_second_moment_is_bit_identical(monkeypatch, V, K, H, B, n_docs, graph):
    """The sparse tile's LDS second-moment variant (the fused-mode default: 64 VGPRs, 4
    workgroups per CU) against the register variant (GFEDNTM_WIN_VL=0): the same state bit
    for bit, the FedAvg pre-scale included."""
    monkeypatch.setenv("GFEDNTM_WIN_VL", "0")
    a = _make(monkeypatch, "0", "prodLDA", V, K, H, B)
    monkeypatch.setenv("GFEDNTM_WIN_VL", "1")
    b = _make(monkeypatch, "0", "prodLDA", V, K, H, B)
    assert a.engine._m.stage_flags & STAGE_WIN_VREG
    assert b.engine._m.stage_flags & STAGE_WIN_SPARSE and not b.engine._m.stage_flags & STAGE_WIN_VREG
    b.model.load_state_dict(a.model.state_dict())
    b.engine.seed = b.engine._m.seed = a.engine.seed
    X = random_csr(n_docs, V, 60, seed=5)
    n_steps = 2 * -(-n_docs // B)
    for tm in (a, b):
        _run(tm, X, n_steps, B, graph)
    _assert_same_state(a, b)
