"""Flat state layout and the FedAvg aggregation (golden test against a numpy
re-statement of the reference server average, server.py:477-487)."""
import numpy as np
import torch

from gfedntm_amd.models.networks import DecoderNetwork
from gfedntm_amd.ops.engine import BETA_PAD
from gfedntm_amd.parallel.aggregator import LocalAggregator, fedavg_weights
from gfedntm_amd.utils.config import DEFAULT_GRADS_TO_SHARE
from gfedntm_amd.utils.flat import ALIGN, FlatState


def _net():
    torch.manual_seed(0)
    return DecoderNetwork(60, 5, "prodLDA", (8, 6), "softplus", 0.2, True)


def test_flat_views_and_shared_prefix():
    m = _net()
    before = {k: v.clone() for k, v in m.state_dict().items()}
    fs = FlatState(m, ["beta", "prior_mean", "inf_net.f_mu.weight", "not_a_key"],
                   transposed=("inf_net.input_layer.weight",))
    # values preserved, parameters are views of the buffer
    for k, v in m.state_dict().items():
        assert torch.equal(v, before[k]), k
    assert m.beta.data_ptr() == fs.view("beta").data_ptr()
    # shared keys come first (state_dict order), unknown keys ignored (B2)
    offs = {k: s.offset for k, s in fs.slots.items()}
    shared = [k for k in ("prior_mean", "beta", "inf_net.f_mu.weight")]
    assert max(offs[k] for k in shared) < min(o for k, o in offs.items() if k not in shared)
    assert fs.shared.numel() >= sum(fs.slots[k].numel for k in shared)
    assert all(s.offset % ALIGN == 0 for s in fs.slots.values())
    # transposed storage: logical [h0, V] view, physical [V, h0]
    w = m.inf_net.input_layer.weight
    assert w.shape == (8, 60) and fs.raw("inf_net.input_layer.weight").shape == (60, 8)
    fs.buffer.mul_(2)
    assert torch.equal(m.beta, 2 * before["beta"])


def test_padded_beta_rows():
    """beta stored with 256-B rows ({"beta": BETA_PAD}, the fused engine's layout): the module sees the [K, V] slice, the
    state_dict / load_state_dict round trip is exact, the pad columns are zero and in the
    slot's storage (param ranges, FedAvg prefix), and rows start on 32-float boundaries."""
    m = _net()                                   # beta [5, 60] -> rows of 64 floats
    before = {k: v.clone() for k, v in m.state_dict().items()}
    fs = FlatState(m, ["beta", "prior_mean"], padded={"beta": BETA_PAD}, shared_last=("beta",))
    s = fs.slots["beta"]
    assert s.ld == 64 and s.numel == 5 * 64 and s.offset % 32 == 0
    assert m.beta.shape == (5, 60) and m.beta.stride() == (64, 1)
    assert m.beta.data_ptr() == fs.buffer[s.offset:].data_ptr()
    for k, v in m.state_dict().items():
        assert torch.equal(v, before[k]), k
    raw = fs.raw("beta")
    assert raw.shape == (5, 64) and torch.count_nonzero(raw[:, 60:]) == 0
    # FedAvg prefix ends with beta's padded storage
    assert fs.n_shared == s.offset + s.numel
    assert any(a <= s.offset and s.offset + s.numel <= b for a, b in fs.param_ranges())
    # a write through the module lands in the strided slot; load_state_dict round trip
    with torch.no_grad():
        m.beta.add_(1.0)
    assert torch.equal(raw[:, :60], before["beta"] + 1) and torch.count_nonzero(raw[:, 60:]) == 0
    m.load_state_dict(before)
    assert torch.equal(m.beta, before["beta"])
    g = torch.zeros_like(fs.buffer)
    assert fs.view_like(g, "beta").shape == (5, 60)


def test_fedavg_golden():
    rng = np.random.default_rng(0)
    n = [120, 80, 200]
    states = [rng.normal(size=1000).astype(np.float32) for _ in n]
    # reference: average of each tensor weighted by nr_samples / total
    ref = sum(s * (ni / sum(n)) for s, ni in zip(states, n))
    flats = [torch.from_numpy(s.copy()) for s in states]
    LocalAggregator(n).average_(flats)
    for f in flats:
        np.testing.assert_allclose(f.numpy(), ref, rtol=1e-6, atol=1e-6)
    # pre-scaled path (what the fused engine feeds): plain sum
    w = fedavg_weights(n)
    flats = [torch.from_numpy(s * wi) for s, wi in zip(states, w)]
    LocalAggregator(n).average_(flats, prescaled=True)
    np.testing.assert_allclose(flats[0].numpy(), ref, rtol=1e-5, atol=1e-6)


def test_default_shared_keys_on_avitm():
    m = _net()
    fs = FlatState(m, DEFAULT_GRADS_TO_SHARE)
    # every float tensor of the AVITM state is shared (adapt_bert keys are absent: B2)
    float_keys = [k for k, v in m.state_dict().items() if v.is_floating_point()]
    assert fs.n_shared >= sum(fs.slots[k].numel for k in float_keys)


def test_fused_shared_tail_orders_the_fedavg_parts():
    """The fused engine's FedAvg parts are contiguous ranges at the end of the shared
    prefix (ops/engine.py fedavg_parts): with topic_model.FUSED_SHARED_LAST a CombinedTM's
    shared state ends [... | adapt_bert.weight, adapt_bert.bias | beta], each part one
    contiguous range; a ProdLDA's ends with beta alone (the adapt_bert keys are absent)."""
    from gfedntm_amd.models.networks import CTMDecoderNetwork
    from gfedntm_amd.models.topic_model import TopicModelBase
    tail = TopicModelBase.FUSED_SHARED_LAST
    torch.manual_seed(0)
    ctm = CTMDecoderNetwork(60, 12, "combined", 5, "prodLDA", (8, 6))
    keys = list(ctm.state_dict().keys())
    fs = FlatState(ctm, keys, transposed=("inf_net.input_layer.weight",), shared_last=tail)
    assert fs.shared_keys[-3:] == list(tail)
    w0 = fs.slots[tail[0]].offset
    b0 = fs.slots["beta"].offset
    rest = [k for k in fs.shared_keys if k not in tail]
    assert max(fs.slots[k].offset + fs.slots[k].numel for k in rest) <= w0 < b0
    assert fs.slots["beta"].offset + fs.slots["beta"].numel == fs.n_shared
    pl = FlatState(_net(), list(_net().state_dict().keys()), shared_last=tail)
    assert pl.shared_keys[-1] == "beta" and tail[0] not in pl.slots
