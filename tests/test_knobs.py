"""The operational environment knobs (docs/DESIGN.md "Stage bits and knobs"): each one read
where docs/DESIGN.md says, with the effect it documents.  The kernel-plan knobs are forced
by the GPU tests that the same table names."""
import socket

import numpy as np
import pytest
import torch

from gfedntm_amd.ops import native


def test_runtime_threads_knob_gives_the_same_csr(monkeypatch):
    """GFEDNTM_RUNTIME_THREADS: the host runtime's worker count (0 = hardware threads);
    any count gives the same vocabulary and CSR (csrc/runtime.cpp)."""
    if not native.tokenizer_available():
        pytest.skip("runtime not built")
    from gfedntm_amd.ops import runtime_abi
    lib = native.runtime()
    rng = np.random.default_rng(3)
    words = ["alpha", "beta", "gamma", "delta", "topic", "model", "federated", "x9", "v2"]
    texts = [" ".join(rng.choice(words, size=rng.integers(1, 30))) for _ in range(2500)]
    out = []
    for n in ("0", "1", "3"):
        monkeypatch.setenv("GFEDNTM_RUNTIME_THREADS", n)
        voc = runtime_abi.local_vocabulary(lib, texts)
        X = runtime_abi.vectorize(lib, texts, voc)
        out.append((voc, X))
    for voc, X in out[1:]:
        assert voc == out[0][0]
        assert (X != out[0][1]).nnz == 0


def test_roctx_knob_turns_markers_off(monkeypatch):
    """GFEDNTM_ROCTX=0: the trace ranges (utils/trace.py) are no-ops."""
    from gfedntm_amd.utils import trace
    monkeypatch.setattr(trace, "_lib", None)
    monkeypatch.setattr(trace, "_tried", False)
    monkeypatch.setenv("GFEDNTM_ROCTX", "0")
    assert trace._roctx() is None and not trace.available()
    ran = False
    with trace.trace_range("knob-test"):      # (a no-op range still runs its body)
        ran = True
    trace.mark("knob-test")
    assert ran


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_allreduce_knob_selects_the_method(monkeypatch):
    """GFEDNTM_ALLREDUCE (rccl | xgmi | auto): the collective aggregator's default method
    (parallel/aggregator.py); an explicit argument wins."""
    import torch.distributed as dist
    from gfedntm_amd.parallel.aggregator import CollectiveAggregator
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0,
                            world_size=1)
    try:
        monkeypatch.setenv("GFEDNTM_ALLREDUCE", "RCCL")
        assert CollectiveAggregator().method == "rccl"
        assert CollectiveAggregator(method="xgmi").method == "xgmi"
        monkeypatch.delenv("GFEDNTM_ALLREDUCE")
        agg = CollectiveAggregator()
        assert agg.method == "auto"
        flat = torch.arange(8, dtype=torch.float32)
        agg.prepare(flat)
        assert agg.active == "rccl"        # (CPU tensors: never the xGMI kernel)
    finally:
        dist.destroy_process_group()


def test_round_batched_knob(monkeypatch):
    """GFEDNTM_ROUND_BATCHED=0: LocalFederation keeps one graph branch per client instead of
    the batched launches (federation/runner.py); the constructor argument wins."""
    from gfedntm_amd.data.synthetic import generate_synthetic
    from gfedntm_amd.federation.data import ClientCorpus
    from gfedntm_amd.federation.runner import LocalFederation
    from gfedntm_amd.utils.config import load_config
    sc = generate_synthetic(vocab_size=200, n_topics=5, n_docs=60, n_nodes=2, frozen_topics=1,
                            nwords=(20, 40), seed=2)
    corpora = [ClientCorpus(synthetic=sc, node=i) for i in range(2)]
    p = dict(load_config().training_params)
    p.update(num_epochs=1, batch_size=16, hidden_sizes=(16, 16), n_components=5)
    kw = dict(max_iters=1, device="cpu", backend="torch", seed=1)
    monkeypatch.setenv("GFEDNTM_ROUND_BATCHED", "0")
    assert LocalFederation(corpora, p, **kw).round_batched is False
    assert LocalFederation(corpora, p, round_batched=True, **kw).round_batched is True
    monkeypatch.delenv("GFEDNTM_ROUND_BATCHED")
    assert LocalFederation(corpora, p, **kw).round_batched is True
