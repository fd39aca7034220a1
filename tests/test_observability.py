"""Liveness watchdog, roctx tracing fallbacks and the JSONL round metrics (CPU)."""
import datetime
import json
import os
import socket
import time

import pytest

import torch.distributed as dist

from gfedntm_amd.parallel.heartbeat import Heartbeat
from gfedntm_amd.utils import trace


def _store():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    return dist.TCPStore("127.0.0.1", port, 2, True, timeout=datetime.timedelta(seconds=30),
                         wait_for_workers=False)


def test_heartbeat_detects_a_dead_peer_and_ignores_a_finished_one():
    store = _store()
    seen = []
    a = Heartbeat(0, 2, store=store, interval=0.05, timeout=0.5, on_failure=seen.append,
                  prefix="t1").start()
    b = Heartbeat(1, 2, store=store, interval=0.05, timeout=0.5, on_failure=lambda d: None,
                  prefix="t1").start()
    time.sleep(0.4)
    assert not seen                       # both alive
    b._stop.set()                         # rank 1 "dies": no more beats, no done flag
    b._thread.join()
    t0 = time.time()
    while not seen and time.time() - t0 < 5:
        time.sleep(0.05)
    assert seen == [[1]]
    a._stop.set()

    seen2 = []
    c = Heartbeat(0, 2, store=store, interval=0.05, timeout=0.5, on_failure=seen2.append,
                  prefix="t2").start()
    d = Heartbeat(1, 2, store=store, interval=0.05, timeout=0.5, on_failure=lambda x: None,
                  prefix="t2").start()
    time.sleep(0.2)
    d.stop()                              # normal completion
    time.sleep(1.2)
    assert not seen2
    c.stop()


def test_heartbeat_exempts_a_busy_peer_from_the_behind_rule():
    """A peer inside long host work (results save) publishes busy: it stays alive as
    long as it beats, even while behind this rank's progress."""
    store = _store()
    seen = []
    a = Heartbeat(0, 2, store=store, interval=0.05, timeout=0.4, on_failure=seen.append,
                  prefix="t3").start()
    b = Heartbeat(1, 2, store=store, interval=0.05, timeout=0.4, on_failure=lambda d: None,
                  prefix="t3").start()
    a.mark(10, 1)                         # rank 0 is ahead
    b.mark(5, 1)
    b.busy(True)                          # rank 1 saves its results for a while
    time.sleep(1.2)
    assert not seen
    b.busy(False)                         # done, but now stuck behind: detected
    t0 = time.time()
    while not seen and time.time() - t0 < 5:
        time.sleep(0.05)
    assert seen == [[1]]
    a._stop.set()
    b._stop.set()


def test_trace_ranges_are_safe_without_a_profiler():
    with trace.trace_range("unit-test"):
        trace.mark("inside")
    w = trace.RoundWindow()
    assert w.close() is None
    w.add(64)
    w.add(32)
    out = w.close()
    assert out["rounds"] == 2 and out["docs"] == 96 and out["docs_per_s"] > 0


def test_cli_writes_jsonl_metrics(tmp_path):
    from gfedntm_amd.cli import main
    main(["--workdir", str(tmp_path), "--min_clients_federation", "2", "--max_iters", "6",
          "--engine", "torch", "--device", "cpu", "--metrics_every", "3",
          "--generate_synthetic", str(tmp_path / "syn.npz")])
    files = [os.path.join(r, f) for r, _, fs in os.walk(tmp_path) for f in fs
             if f.startswith("metrics_") and f.endswith(".jsonl")]
    assert len(files) == 1
    rows = [json.loads(l) for l in open(files[0])]
    windows = [r for r in rows if r["event"] == "window"]
    end = [r for r in rows if r["event"] == "train_end"]
    assert [w["round"] for w in windows] == [3, 6] and len(end) == 1
    assert end[0]["rounds"] == 6 and end[0]["docs_per_s"] > 0
    assert all(w["docs"] > 0 and w["loss"] > 0 for w in windows)


def _hang_worker(rank, world, port, tmp):
    import os as _os
    import time as _time
    _os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                       WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world,
                            timeout=datetime.timedelta(seconds=600))
    from gfedntm_amd.data.synthetic import generate_synthetic
    from gfedntm_amd.federation import client as client_mod
    from gfedntm_amd.federation.data import ClientCorpus
    from gfedntm_amd.federation.runner import run_distributed
    from gfedntm_amd.utils.config import load_config
    orig = client_mod.FederatedClient.local_step

    def local_step(self, it):
        if rank == 1 and it == 3:
            _time.sleep(600)                  # the main thread hangs; its heartbeat lives on
        return orig(self, it)

    client_mod.FederatedClient.local_step = local_step
    params = dict(load_config().training_params)
    params.update(num_epochs=2, batch_size=16, hidden_sizes=(16, 16), n_components=5)
    sc = generate_synthetic(vocab_size=60, n_topics=5, n_docs=30, n_nodes=2, frozen_topics=1,
                            nwords=(10, 20), seed=2)
    run_distributed(ClientCorpus(synthetic=sc, node=rank), params, max_iters=50,
                    backend="torch", heartbeat_timeout=10.0)


def test_hung_peer_aborts_the_waiting_rank(tmp_path):
    """A rank whose training loop hangs (process alive) is detected by the waiting
    rank, which aborts (exit code 3) instead of blocking in the collective."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ps = [ctx.Process(target=_hang_worker, args=(r, 2, port, str(tmp_path))) for r in range(2)]
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


def _kill_worker(rank, world, port):
    import os as _os
    _os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                       WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world,
                            timeout=datetime.timedelta(seconds=600))
    from gfedntm_amd.data.synthetic import generate_synthetic
    from gfedntm_amd.federation import client as client_mod
    from gfedntm_amd.federation.data import ClientCorpus
    from gfedntm_amd.federation.runner import run_distributed
    from gfedntm_amd.utils.config import load_config
    orig = client_mod.FederatedClient.local_step

    def local_step(self, it):
        if rank == 1 and it == 3:
            _os._exit(9)                      # the process dies mid-round
        return orig(self, it)

    client_mod.FederatedClient.local_step = local_step
    params = dict(load_config().training_params)
    params.update(num_epochs=2, batch_size=16, hidden_sizes=(16, 16), n_components=5)
    sc = generate_synthetic(vocab_size=60, n_topics=5, n_docs=30, n_nodes=world, frozen_topics=1,
                            nwords=(10, 20), seed=2)
    run_distributed(ClientCorpus(synthetic=sc, node=rank), params, max_iters=50,
                    backend="torch", heartbeat_timeout=10.0)


def test_killed_peer_ends_the_surviving_rank():
    """a rank killed mid-round makes the surviving rank stop with an error
    (peer connection closed or liveness timeout) instead of hanging."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ps = [ctx.Process(target=_kill_worker, args=(r, 2, port)) for r in range(2)]
    for p in ps:
        p.start()
    ps[1].join(120)
    ps[0].join(120)
    try:
        assert ps[1].exitcode == 9, ps[1].exitcode
        assert ps[0].exitcode not in (None, 0), ps[0].exitcode    # ended, with an error
    finally:
        for p in ps:
            if p.is_alive():
                p.kill()
            p.join(10)


@pytest.mark.parametrize("n_clients", [2, 4])
def test_distributed_windows_carry_loss_kl_rl(tmp_path, n_clients):
    """The production runner (run_distributed over gloo ranks: one client per rank, and
    two per rank) writes loss, KL and RL into every JSONL window (reference
    federated_avitm.py:109 logs the minibatch loss), and the loss equals KL + RL (AVITM,
    KL weight 1: loss_hist is the batch sum, the terms are batch means)."""
    from gfedntm_amd.cli import main
    main(["--backend", "gloo", "--workdir", str(tmp_path), "--min_clients_federation",
          str(n_clients), "--nproc", "2", "--max_iters", "6", "--engine", "torch",
          "--device", "cpu", "--metrics_every", "3", "--log_every", "2",
          "--generate_synthetic", str(tmp_path / "syn.npz")])
    files = [os.path.join(r, f) for r, _, fs in os.walk(tmp_path) for f in fs
             if f.startswith("metrics_") and f.endswith(".jsonl")]
    assert files
    windows = [json.loads(l) for f in files for l in open(f)]
    windows = [w for w in windows if w["event"] == "window"]
    assert windows and {w["round"] for w in windows} == {3, 6}
    for w in windows:
        assert {"loss", "kl", "rl", "docs", "ms_per_round"} <= set(w), w
        assert w["kl"] > 0 and w["rl"] > 0 and w["loss"] > w["rl"]
