"""Gradient aggregation (``--agg grads``, SURVEY.md §2.4 "classic synchronous DP",
optional, not the reference semantics): every client computes its minibatch
gradient, the sample-weighted average is all-reduced, every client applies the same
optimizer step (replicas stay identical), batch-norm running statistics averaged."""
import os
import socket

import numpy as np
import pytest
import torch

from gfedntm_amd.federation.runner import LocalFederation
from gfedntm_amd.models.engine import make_optimizer
from gfedntm_amd.models.networks import kl_terms, reconstruction_terms
from tests.test_federation import _corpora, _params


def test_grads_mode_matches_synchronous_data_parallel():
    fed = LocalFederation(_corpora(), _params(), max_iters=5, device="cpu", backend="torch",
                          seed=2, agg="grads")
    sd0 = {k: v.clone() for k, v in fed.clients[0].tm.model.state_dict().items()}
    from gfedntm_amd.models.networks import DecoderNetwork
    models = []
    for c in fed.clients:
        m = DecoderNetwork(c.tm.input_size, 5, "prodLDA", (16, 16), "softplus", 0.2, True)
        m.load_state_dict(sd0)
        models.append((m, make_optimizer(m.parameters(), "adam", 2e-3, 0.99)))
    n = np.array([c.n_docs for c in fed.clients], dtype=np.float64)
    w = n / n.sum()
    fed.run()
    # every client's noise comes from its own stream (seeded with its client seed)
    states = [torch.Generator().manual_seed(2 + c.id).get_state() for c in fed.clients]
    for it in range(5):
        grads = []
        for i, ((m, opt), c) in enumerate(zip(models, fed.clients)):
            ids = torch.from_numpy(c.plan.batch(it).astype(np.int64))
            x = c.data.dense_rows(ids)
            m.train()
            opt.zero_grad()
            with torch.random.fork_rng(devices=[]):
                torch.set_rng_state(states[i])
                pm, pv, mu, var, lv, wd = m(x)
                states[i] = torch.get_rng_state()
            loss = (kl_terms(pm, pv, mu, var, lv, 5) + reconstruction_terms(x, wd)).sum()
            loss.backward()
            grads.append({k: p.grad.clone() for k, p in m.named_parameters()})
        avg_g = {k: sum(wi * g[k] for wi, g in zip(w, grads)) for k in grads[0]}
        for m, opt in models:
            for k, p in m.named_parameters():
                p.grad.copy_(avg_g[k])
            opt.step()
        bufs = {k: sum(wi * mm.state_dict()[k] for wi, (mm, _) in zip(w, models))
                for k, v in models[0][0].named_buffers() if v.is_floating_point()}
        for m, _ in models:
            for k, v in bufs.items():
                m.state_dict()[k].copy_(v)
    for (m, _), c in zip(models, fed.clients):
        for k, v in m.state_dict().items():
            torch.testing.assert_close(c.tm.model.state_dict()[k].to(v.dtype), v, rtol=1e-5,
                                       atol=1e-6, msg=lambda s: f"{k}: {s}")
    # replicas identical, optimizer states identical
    a = fed.clients[0]
    for o in fed.clients[1:]:
        assert torch.equal(o.tm.flat.buffer, a.tm.flat.buffer)


def _dist_worker(rank, world, port, q):
    import torch.distributed as dist
    from gfedntm_amd.federation.runner import run_distributed
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        out = run_distributed(_corpora(world)[rank], _params(), max_iters=4, backend="torch",
                              seed=0, agg_mode="grads")
        q.put((rank, out["client"].tm.flat.buffer.numpy().copy()))
    finally:
        dist.destroy_process_group()


def test_grads_mode_gloo_two_ranks():
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_dist_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=240) for _ in procs), key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert np.isfinite(res[0][1]).all()
    np.testing.assert_array_equal(res[0][1], res[1][1])    # whole state, incl. non-shared


def test_grads_mode_rejected_on_grpc(tmp_path):
    from gfedntm_amd.cli import main
    with pytest.raises(SystemExit):
        main(["--backend", "grpc", "--agg", "grads", "--workdir", str(tmp_path)])


@pytest.mark.gpu
@pytest.mark.parametrize("model_type", ["avitm", "ctm"])
def test_fused_grads_mode_one_round(model_type):
    """Fused engine: kernels in gradient mode, all-reduce of the pre-scaled gradients,
    then the generic Adam: after round 0 every replica equals the Adam step
    p - lr * g / (|g| + eps) (t = 1) on the averaged gradient."""
    params = _params(hidden_sizes=(32, 32), n_components=8)
    corpora = _corpora(2)
    if model_type == "ctm":
        for i, c in enumerate(corpora):
            c.embeddings = np.random.default_rng(i).standard_normal(
                (c.n_docs, 64)).astype(np.float32)
        params.update(contextual_size=64)
    fed = LocalFederation(corpora, params, model_type=model_type, max_iters=3, device="cuda",
                          backend="fused", seed=1, agg="grads")
    cs = fed.clients
    p0 = cs[0].tm.flat.buffer.clone()
    for c in cs:
        c.local_step(0)
    g = sum(c.shared_grads.clone() for c in cs)
    fed.agg.average_([c.shared_grads for c in cs], prescaled=True)
    for c in cs:
        c.apply_step(0)
    torch.cuda.synchronize()
    lr, eps = cs[0].tm.engine.lr, cs[0].tm.engine.eps
    mask = cs[0].tm.flat.param_mask()[: g.numel()].bool()
    want = p0[: g.numel()] - lr * g / (g.abs() + eps)
    got = cs[1].tm.flat.buffer[: g.numel()]
    torch.testing.assert_close(got[mask], want[mask], rtol=1e-5, atol=1e-6)
    assert torch.equal(cs[0].tm.flat.buffer[mask.nonzero()[:, 0]], got[mask])
    # whole rounds through run(): replicas stay identical, loss finite
    fed.run()
    torch.cuda.synchronize()
    assert torch.equal(cs[0].tm.flat.buffer, cs[1].tm.flat.buffer)
    assert torch.isfinite(cs[0].tm.engine.loss_hist).all()
