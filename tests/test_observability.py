"""Liveness watchdog, roctx tracing fallbacks and the JSONL round metrics (CPU)."""
import datetime
import json
import os
import socket
import time

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
