"""The production CLI on the GPU data plane: ``main.py --backend rccl`` (reference main.py:
178-291 -- flags, synthetic source, outputs) through ``run_collective``: the spawned rank
initialises the "nccl" (RCCL) process group with ``device_id`` and runs
``_rank_main`` -> ``run_distributed`` with the fused engine.

* one client on one rank: the client's ``model_1_<date>.npz`` (betas / thetas / topics in
  the reference layout), the server's ``global_model_<date>.npz`` (betas only), the
  reference log lines;
* ``--min_clients_federation 3 --nproc 1``: one RCCL rank hosting three clients (batched
  steps + in-rank fold), every client saving its results.
"""
import configparser
import datetime
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _config(tmp_path) -> str:
    cp = configparser.ConfigParser()
    cp.read(os.path.join(ROOT, "config", "dft_params.cf"))
    cp.set("ntms", "num_epochs", "1")
    cp.set("ntms", "n_components", "10")
    path = str(tmp_path / "cfg.cf")
    with open(path, "w") as f:
        cp.write(f)
    return path


def _run(tmp_path, n_clients: int):
    src = str(tmp_path / "syn.npz")
    if not os.path.exists(src):
        from gfedntm_amd.data.synthetic import generate_synthetic
        generate_synthetic(vocab_size=800, n_topics=10, n_docs=150, n_nodes=3, frozen_topics=2,
                           nwords=(40, 80), seed=2).save_counts_npz(src)
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "main.py"), "--backend", "rccl",
                        "--nproc", "1", "--min_clients_federation", str(n_clients),
                        "--max_iters", "12", "--source", src, "--workdir", str(tmp_path),
                        "--config", _config(tmp_path), "--heartbeat_timeout", "60"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-4000:]
    return p


def test_cli_rccl_one_client_writes_reference_outputs(tmp_path):
    from gfedntm_amd.eval.export import load_model_npz
    p = _run(tmp_path, 1)
    stamp = datetime.datetime.now().strftime("%Y%m%d")
    out = tmp_path / "static" / "output_models"
    z = load_model_npz(str(out / "client1" / f"model_1_{stamp}.npz"))
    assert z["betas"].shape[0] == 10 and np.allclose(z["betas"].sum(1), 1, atol=1e-4)
    assert z["thetas"].shape == (150, 10) and np.allclose(z["thetas"].sum(1), 1)
    assert z["topics"].shape == (10, 10)
    g = load_model_npz(str(out / "server" / f"global_model_{stamp}.npz"))
    assert set(g) == {"betas", "ntopics"}
    logs = (tmp_path / "static" / "logs" / "client1" / f"logs_{stamp}.txt").read_text()
    assert "Epoch: [1/1]" in logs and "Saving model" in logs
    # the ground truth of the synthetic source is scored at the save (reference
    # evaluate_synthetic_model)
    assert "evaluados correctamente" in logs and "doc similarity" in logs
    assert "Global vocabulary agreed" in p.stdout + p.stderr + logs


def test_cli_rccl_three_clients_on_one_rank(tmp_path):
    from gfedntm_amd.eval.export import load_model_npz
    _run(tmp_path, 3)
    stamp = datetime.datetime.now().strftime("%Y%m%d")
    out = tmp_path / "static" / "output_models"
    for i in (1, 2, 3):
        z = load_model_npz(str(out / f"client{i}" / f"model_{i}_{stamp}.npz"))
        assert z["thetas"].shape == (150, 10)
    assert os.path.exists(out / "server" / f"global_model_{stamp}.npz")
