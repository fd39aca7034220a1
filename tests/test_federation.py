"""Federation protocol on CPU: reference round semantics (golden simulation),
checkpoint / resume, gloo multi-process, CLI."""
import os

import numpy as np
import pytest
import torch

from gfedntm_amd.data.synthetic import generate_synthetic
from gfedntm_amd.eval.export import load_model_npz
from gfedntm_amd.federation.data import ClientCorpus, load_client_corpus
from gfedntm_amd.federation.runner import LocalFederation
from gfedntm_amd.models.engine import make_optimizer
from gfedntm_amd.models.networks import kl_terms, reconstruction_terms
from gfedntm_amd.utils.config import load_config


def _params(**kw):
    p = dict(load_config().training_params)
    p.update(num_epochs=2, batch_size=16, hidden_sizes=(16, 16), n_components=5)
    p.update(kw)
    return p


def _corpora(n=3, seed=1):
    sc = generate_synthetic(vocab_size=120, n_topics=5, n_docs=40, n_nodes=n, frozen_topics=2,
                            nwords=(15, 30), seed=seed)
    return [ClientCorpus(synthetic=sc, node=i) for i in range(n)]


def test_rounds_match_reference_semantics():
    """Every round: each client one local Adam step on its own minibatch, then the
    sample-weighted average of the shared state (server.py:477-487) -- re-stated
    with plain torch modules and compared tensor by tensor."""
    fed = LocalFederation(_corpora(), _params(), max_iters=6, device="cpu", backend="torch", seed=2)
    sds = [{k: v.clone() for k, v in c.tm.model.state_dict().items()} for c in fed.clients]
    # golden simulation
    from gfedntm_amd.models.networks import DecoderNetwork
    models = []
    for c, sd in zip(fed.clients, sds):
        m = DecoderNetwork(c.tm.input_size, 5, "prodLDA", (16, 16), "softplus", 0.2, True)
        m.load_state_dict(sd)
        models.append((m, make_optimizer(m.parameters(), "adam", 2e-3, 0.99)))
    n = np.array([c.n_docs for c in fed.clients], dtype=np.float64)
    w = n / n.sum()
    fed.run()
    # each client draws its noise from its own stream seeded with its client seed (as
    # the reference's clients, one process each, do)
    states = [torch.Generator().manual_seed(2 + c.id).get_state() for c in fed.clients]
    for it in range(6):
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
            opt.step()
        avg = {}
        for k, v in models[0][0].state_dict().items():
            if v.is_floating_point():
                avg[k] = sum(wi * mm.state_dict()[k] for wi, (mm, _) in zip(w, models))
        for m, _ in models:
            sd = m.state_dict()
            for k, v in avg.items():
                sd[k].copy_(v)
    for (m, _), c in zip(models, fed.clients):
        for k, v in m.state_dict().items():
            torch.testing.assert_close(c.tm.model.state_dict()[k].to(v.dtype), v, rtol=1e-5,
                                       atol=1e-6, msg=lambda s: f"{k}: {s}")


def test_outputs_and_bookkeeping(tmp_path):
    fed = LocalFederation(_corpora(2), _params(num_epochs=1), max_iters=5, device="cpu",
                          backend="torch", save_client=str(tmp_path / "client"),
                          save_server=str(tmp_path / "server"), seed=0, stamp="20240101")
    fed.run()
    c = fed.clients[0]
    assert c.current_epoch >= 1 and c.samples_processed == sum(c.plan.size[:5])
    z = load_model_npz(str(tmp_path / "client1" / "model_1_20240101.npz"))
    assert z["betas"].shape == (5, len(fed.terms)) and z["thetas"].shape == (40, 5)
    assert np.allclose(z["thetas"].sum(1), 1) and z["topics"].shape == (5, 10)
    g = load_model_npz(str(tmp_path / "server" / "global_model_20240101.npz"))
    assert set(g) == {"betas", "ntopics"}
    # all clients hold the same (averaged) state
    for o in fed.clients[1:]:
        assert torch.equal(o.shared, c.shared)


def test_checkpoint_resume_is_exact(tmp_path):
    kw = dict(max_iters=6, device="cpu", backend="torch", seed=4)
    torch.manual_seed(11)
    full = LocalFederation(_corpora(), _params(), **kw)
    full.run()
    torch.manual_seed(11)
    a = LocalFederation(_corpora(), _params(), checkpoint_dir=str(tmp_path), checkpoint_every=3,
                        **dict(kw, max_iters=3))
    a.run()
    b = LocalFederation(_corpora(), _params(), checkpoint_dir=str(tmp_path), checkpoint_every=3,
                        **kw)
    assert b.round == 3
    b.run()
    for cf, cb in zip(full.clients, b.clients):
        torch.testing.assert_close(cb.shared, cf.shared, rtol=0, atol=0)
        assert cb.current_epoch == cf.current_epoch and cb.samples_processed == cf.samples_processed


def _dist_worker(rank, world, port, tmp, q):
    import torch.distributed as dist
    from gfedntm_amd.federation.runner import run_distributed
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        corpus = _corpora(world)[rank]
        out = run_distributed(corpus, _params(), max_iters=5, backend="torch", seed=0,
                              save_client=os.path.join(tmp, "client"),
                              save_server=os.path.join(tmp, "server"), stamp="20240101")
        q.put((rank, out["client"].shared.numpy().copy(), out["rounds"]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_gloo_ranks(tmp_path, world):
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_dist_worker, args=(r, world, port, str(tmp_path), q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=240) for _ in procs), key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(r[2] == 5 for r in res)
    for r in res[1:]:
        np.testing.assert_array_equal(res[0][1], r[1])        # identical averaged state
    assert os.path.exists(tmp_path / f"client{world}" / f"model_{world}_20240101.npz")
    assert os.path.exists(tmp_path / "server" / "global_model_20240101.npz")


def test_cli_local(tmp_path):
    from gfedntm_amd.cli import main
    out = main(["--workdir", str(tmp_path), "--min_clients_federation", "2", "--max_iters", "4",
                "--engine", "torch", "--device", "cpu",
                "--generate_synthetic", str(tmp_path / "syn.npz")])
    assert out["rounds"] == 4
    found = [f for _, _, fs in os.walk(tmp_path) for f in fs]
    assert any(f.startswith("global_model_") for f in found)
    assert any(f.startswith("logs_") for f in found)


def test_load_client_corpus(tmp_path):
    sc = generate_synthetic(vocab_size=50, n_topics=3, n_docs=10, n_nodes=2, frozen_topics=1,
                            nwords=(5, 9), seed=0)
    p = str(tmp_path / "c.npz")
    sc.save_counts_npz(p)
    c = load_client_corpus("synthetic", p, 2)
    assert c.n_docs == 10 and c.ground_truth_thetas.shape == (10, 3)
    ref = str(tmp_path / "ref.npz")
    sc.save_npz(ref)                                   # reference schema (object arrays)
    with pytest.raises(ValueError):
        load_client_corpus("synthetic", ref, 1)
    c2 = load_client_corpus("synthetic", ref, 1, allow_pickle=True)
    assert c2.n_docs == 10 and c2.local_terms() == ClientCorpus(synthetic=sc, node=0).local_terms()
    import pandas as pd
    df = pd.DataFrame({"bow_text": ["alpha beta gamma", "beta delta", "zeta eta"],
                       "fos": ["cs", "cs", "bio"], "embeddings": ["0.1 0.2", "0.3 0.4", "1 2"]})
    pq = str(tmp_path / "r.parquet")
    df.to_parquet(pq)
    r = load_client_corpus("real", pq, 1, fos="cs")
    assert r.n_docs == 2 and r.embeddings.shape == (2, 2) and "gamma" in r.local_terms()


def test_assign_clients_partitions():
    from gfedntm_amd.federation.hierarchical import assign_clients
    assert assign_clients(16, 2) == [list(range(1, 9)), list(range(9, 17))]
    assert assign_clients(5, 2) == [[1, 2, 3], [4, 5]]
    assert assign_clients(8, 8) == [[i] for i in range(1, 9)]
    with pytest.raises(ValueError):
        assign_clients(2, 3)


def _multi_worker(rank, world, port, tmp, n_clients, q):
    import torch.distributed as dist
    from gfedntm_amd.federation.hierarchical import assign_clients, run_distributed_multi
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ids = assign_clients(n_clients, world)[rank]
        corpora = _corpora(n_clients)
        torch.manual_seed(11)
        out = run_distributed_multi([corpora[i - 1] for i in ids], ids, _params(), max_iters=5,
                                    backend="torch", seed=0,
                                    save_client=os.path.join(tmp, "client"),
                                    save_server=os.path.join(tmp, "server"), stamp="20240101")
        q.put((rank, [c.shared.numpy().copy() for c in out["clients"]], out["rounds"],
               [c.id for c in out["clients"]]))
    except Exception:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, traceback.format_exc(), None, None))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n_clients,world", [(4, 2), (5, 2), (40, 2)])
def test_more_clients_than_ranks_matches_grouped_golden(tmp_path, n_clients, world):
    """N clients on R < N gloo ranks (contiguous blocks per rank, hierarchical FedAvg)
    equal the in-process federation with the same grouping; every client of every rank
    ends holding the same state, and every client's results are written.  40 clients on
    2 ranks: 20 per rank, beyond the old 16-buffer limit of the in-rank fold."""
    import socket
    import torch.multiprocessing as mp
    from gfedntm_amd.federation.hierarchical import assign_clients
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_multi_worker, args=(r, world, port, str(tmp_path), n_clients, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=240) for _ in procs), key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
    for r in res:
        assert r[2] == 5, r[1]
    ids = [i for r in res for i in r[3]]
    assert ids == list(range(1, n_clients + 1))
    torch.manual_seed(11)
    groups = [len(b) for b in assign_clients(n_clients, world)]
    gold = LocalFederation(_corpora(n_clients), _params(), max_iters=5, device="cpu",
                           backend="torch", seed=0, groups=groups)
    gold.run()
    g = gold.clients[0].shared.numpy()
    for r in res:
        for sh in r[1]:
            np.testing.assert_array_equal(sh, g)
    for i in range(1, n_clients + 1):
        assert os.path.exists(tmp_path / f"client{i}" / f"model_{i}_20240101.npz")
    assert os.path.exists(tmp_path / "server" / "global_model_20240101.npz")


def test_cli_more_clients_than_ranks(tmp_path):
    """main.py --backend gloo --min_clients_federation 4 --nproc 2: two ranks host two
    clients each (hierarchical FedAvg); every client saves its results, rank 0 the
    global model."""
    from gfedntm_amd.cli import main
    main(["--backend", "gloo", "--workdir", str(tmp_path), "--min_clients_federation", "4",
          "--nproc", "2", "--max_iters", "4", "--engine", "torch", "--device", "cpu",
          "--generate_synthetic", str(tmp_path / "syn.npz")])
    found = [f for _, _, fs in os.walk(tmp_path) for f in fs]
    assert any(f.startswith("global_model_") for f in found)
    for i in range(1, 5):
        assert any(f.startswith(f"model_{i}_") for f in found), (i, found)


def _multi_hang_worker(rank, world, port):
    import datetime
    import time as _time
    import torch.distributed as dist
    from gfedntm_amd.federation import client as client_mod
    from gfedntm_amd.federation.hierarchical import assign_clients
    from gfedntm_amd.federation.runner import run_distributed
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world,
                            timeout=datetime.timedelta(seconds=600))
    orig = client_mod.FederatedClient.local_step

    def local_step(self, it):
        if rank == 1 and it == 3 and self.id == 3:
            _time.sleep(600)                  # the main thread hangs; its heartbeat lives on
        return orig(self, it)

    client_mod.FederatedClient.local_step = local_step
    ids = assign_clients(4, world)[rank]
    corpora = _corpora(4)
    run_distributed([corpora[i - 1] for i in ids], _params(), max_iters=50, backend="torch",
                    heartbeat_timeout=10.0, client_ids=ids)


def test_heartbeat_with_more_clients_than_ranks():
    """--heartbeat_timeout with N > R (2 clients per rank): a rank whose loop hangs in one
    of its clients' steps is detected by its peer, which aborts (exit code 3) instead of
    blocking in the collective -- the same watchdog as one client per rank."""
    import socket
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ps = [ctx.Process(target=_multi_hang_worker, args=(r, 2, port)) for r in range(2)]
    for p in ps:
        p.start()
    ps[0].join(120)
    try:
        assert ps[0].exitcode == 3, ps[0].exitcode
    finally:
        for p in ps:
            if p.is_alive():
                p.kill()
            p.join(10)


def test_federated_synthetic_evaluation_is_logged(tmp_path, caplog):
    """On synthetic sources every client scores its saved model against the generator's
    ground truth (reference federated_avitm.py:152-193): TSS over the generator vocabulary
    and DSS over its own documents, logged with the reference's lines and recomputable
    from the saved npz."""
    import logging
    from gfedntm_amd.eval.metrics import betas_to_ground_truth_vocab, dss, tss
    corpora = _corpora(2)
    log = logging.getLogger("tests.synthetic_eval")      # propagates to caplog
    log.propagate = True
    with caplog.at_level(logging.INFO):
        fed = LocalFederation(corpora, _params(num_epochs=1), max_iters=5, device="cpu",
                              backend="torch", save_client=str(tmp_path / "client"), seed=0,
                              stamp="20240101", logger=log)
        fed.run()
    assert "evaluados correctamente" in caplog.text and "doc similarity" in caplog.text
    for c, corp in zip(fed.clients, corpora):
        ev = c.synthetic_eval
        assert ev is not None and ev["tss"] > 0 and ev["dss"] >= 0
        z = load_model_npz(str(tmp_path / f"client{c.id}" / f"model_{c.id}_20240101.npz"))
        gt_th, gt_b = corp.ground_truth()
        b = betas_to_ground_truth_vocab(z["betas"], c.dataset.idx2token, gt_b.shape[1])
        assert abs(tss(b, gt_b) - ev["tss"]) < 1e-9
        assert abs(dss(gt_th, z["thetas"]) - ev["dss"]) < 1e-9
