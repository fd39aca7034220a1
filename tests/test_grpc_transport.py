"""gRPC transport: wire schema parity with the reference federated.proto, codecs,
and a loopback federation (server + 2 clients on 127.0.0.1, CPU)."""
import os
import re
import socket
import threading

import numpy as np
import pytest
import torch

from gfedntm_amd.federation import wire
from gfedntm_amd.federation.wire import pb

grpc = pytest.importorskip("grpc")

REF_PROTO = "/root/reference/src/protos/federated.proto"


def _walk(desc, prefix=""):
    for m in desc.message_types_by_name.values() if hasattr(desc, "message_types_by_name") \
            else desc.nested_types:
        name = prefix + m.name
        yield name, m
        yield from _walk(m, name + ".")


@pytest.mark.skipif(not os.path.exists(REF_PROTO), reason="reference proto not present")
def test_schema_matches_reference_proto():
    """Every `type name = N;` line of the reference proto has the same number here."""
    text = open(REF_PROTO).read()
    ours = {}
    for name, m in _walk(wire._FILE):
        for f in m.fields:
            ours.setdefault(f.name, set()).add(f.number)
    fields = re.findall(r"^\s*(?:optional\s+|repeated\s+)?[\w.]+\s+(\w+)\s*=\s*(\d+)\s*;", text, re.M)
    assert len(fields) > 60
    for fname, num in fields:
        if fname.isupper():          # enum values
            assert wire.MessageType[fname] == int(num)
            continue
        assert int(num) in ours.get(fname, set()), (fname, num)
    for svc in re.findall(r"service\s+(\w+)", text):
        assert svc in wire.SERVICES
    for rpc, req, resp in re.findall(r"rpc\s+(\w+)\s*\(\s*(\w+)\s*\)\s*returns\s*\(\s*(\w+)", text):
        assert any(wire.SERVICES[s].get(rpc) == (req, resp) for s in wire.SERVICES), rpc


def test_codecs_roundtrip():
    from gfedntm_amd.models.networks import DecoderNetwork
    m = DecoderNetwork(30, 4, "prodLDA", (8, 8), "softplus", 0.2, True)
    sd = m.state_dict()
    mu = pb.ModelUpdate.FromString(wire.model_update_from_state(sd, 3).SerializeToString())
    assert mu.HasField("inf_net_hiddens_l00_weight") and mu.HasField("inf_net_hiddens_l_00_bias")
    back = wire.state_from_model_update(mu)
    assert set(back) == set(sd)
    for k in sd:
        assert back[k].dtype == sd[k].dtype and torch.equal(back[k], sd[k]), k
    opt = torch.optim.Adam(m.parameters(), lr=2e-3, betas=(0.99, 0.99))
    m(torch.rand(5, 30) * 3)[2].sum().backward()
    opt.step()
    osd = opt.state_dict()
    rt = wire.adam_state_dict_from_update(
        pb.OptUpdate.FromString(wire.adam_update_from_state_dict(osd).SerializeToString()))
    assert set(rt["state"]) == set(osd["state"])
    for i, st in osd["state"].items():
        assert torch.equal(rt["state"][i]["exp_avg"], st["exp_avg"])
        assert float(rt["state"][i]["step"]) == float(st["step"])
    params = {"n_components": 5, "hidden_sizes": (16, 16), "activation": "softplus",
              "lr": 2e-3, "learn_priors": True, "topic_prior_mean": None}
    got = wire.params_from_dictionary(pb.Dictionary.FromString(
        wire.dictionary_from_params(params).SerializeToString()))
    assert got["hidden_sizes"] == (16, 16) and got["learn_priors"] is True
    assert got["topic_prior_mean"] is None and got["activation"] == "softplus"
    assert abs(got["lr"] - 2e-3) < 1e-9 and got["n_components"] == 5


def test_weighted_average_reference_rule():
    from gfedntm_amd.federation.grpc_transport import weighted_average
    a = {"w": np.array([1.0, 2.0], np.float32), "n": np.array(3, np.int64)}
    b = {"w": np.array([3.0, 6.0], np.float32), "n": np.array(5, np.int64)}
    out = weighted_average([a, b], [1, 3])
    np.testing.assert_allclose(out["w"], [2.5, 5.0])
    assert out["n"].dtype == np.int64 and int(out["n"]) == 4


def _free_base(k):
    for _ in range(50):
        base = np.random.randint(20000, 60000)
        ok = True
        for p in range(base, base + k + 1):
            with socket.socket() as s:
                try:
                    s.bind(("127.0.0.1", p))
                except OSError:
                    ok = False
                    break
        if ok:
            return base
    raise RuntimeError("no free ports")


def test_loopback_federation(tmp_path):
    from gfedntm_amd.data.synthetic import generate_synthetic
    from gfedntm_amd.eval.export import load_model_npz
    from gfedntm_amd.federation.data import ClientCorpus
    from gfedntm_amd.federation.grpc_transport import FederationServicer, run_client, serve
    from gfedntm_amd.utils.config import load_config
    params = dict(load_config().training_params)
    params.update(num_epochs=1, batch_size=16, hidden_sizes=(16, 16), n_components=5)
    sc = generate_synthetic(vocab_size=100, n_topics=5, n_docs=30, n_nodes=2, frozen_topics=2,
                            nwords=(15, 30), seed=3)
    corpora = [ClientCorpus(synthetic=sc, node=i) for i in range(2)]
    base = _free_base(2)
    iters = 5
    svc = FederationServicer(params, "avitm", 2, iters, client_host="127.0.0.1", base_port=base,
                             save_server=str(tmp_path / "server" / ""), wait_timeout=120)
    server = serve(svc, base)
    clients, errors = {}, []

    def run(i):
        try:
            clients[i] = run_client(corpora[i - 1], i, f"127.0.0.1:{base}", base + i,
                                    backend="torch", device="cpu", seed=0,
                                    save_client=str(tmp_path / "client"), timeout=120,
                                    max_iters=iters)
        except BaseException as e:  # pragma: no cover - surfaced below
            errors.append(e)

    ts = [threading.Thread(target=run, args=(i,)) for i in (1, 2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(180)
    assert svc.done.wait(10)
    server.stop(0)
    assert not errors, errors
    assert svc.error is None
    assert svc.rounds == iters
    # every client holds the server's aggregate of the last round
    for c in clients.values():
        sd = c.tm.model.state_dict()
        for k, v in svc.aggregated.items():
            np.testing.assert_allclose(sd[k].numpy(), v, rtol=0, atol=1e-6, err_msg=k)
        assert c.results_saved and c.current_epoch >= 1
    # W0 came from the server: identical vocab on both clients
    assert clients[1].tm.input_size == clients[2].tm.input_size == len(svc.terms)
    # outputs: two client npz + the global betas
    files = [os.path.join(r, f) for r, _, fs in os.walk(tmp_path) for f in fs if f.endswith(".npz")]
    assert len(files) == 3, files
    for f in files:
        out = load_model_npz(f)
        assert out["betas"].shape == (5, len(svc.terms))


def test_cli_grpc_processes(tmp_path):
    """``main.py --backend grpc``: server (--id 0) and two clients as separate processes."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    from gfedntm_amd.data.synthetic import generate_synthetic
    syn = str(tmp_path / "syn.npz")
    generate_synthetic(vocab_size=80, n_topics=5, n_docs=20, n_nodes=2, frozen_topics=2,
                       nwords=(10, 20), seed=5).save_counts_npz(syn)
    base = _free_base(2)
    common = ["--backend", "grpc", "--workdir", str(tmp_path), "--min_clients_federation", "2",
              "--max_iters", "3", "--engine", "torch", "--device", "cpu", "--source", syn,
              "--server_port", str(base), "--base_port", str(base),
              "--server_address", f"127.0.0.1:{base}"]
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    procs = [subprocess.Popen([sys.executable, os.path.join(root, "main.py"), "--id", str(i)]
                              + common, cwd=str(tmp_path), env=env,
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
             for i in (0, 1, 2)]
    outs = []
    try:
        for p in procs:
            outs.append(p.communicate(timeout=240)[0].decode(errors="replace"))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    for p, o in zip(procs, outs):
        assert p.returncode == 0, o[-3000:]
    found = [f for _, _, fs in os.walk(tmp_path) for f in fs]
    assert any(f.startswith("global_model_") for f in found)
    assert sum(f.startswith("model_") for f in found) == 2


def test_client_servicer_is_idempotent_per_round():
    """A retried getGradient / sendAggregatedTensor (after a deadline) must not train
    or apply twice."""
    from gfedntm_amd.data.synthetic import generate_synthetic
    from gfedntm_amd.data.vocab import vocabulary_dict
    from gfedntm_amd.federation.client import FederatedClient
    from gfedntm_amd.federation.data import ClientCorpus
    from gfedntm_amd.federation.grpc_transport import ClientServicer
    from gfedntm_amd.federation.runner import build_dataset, make_topic_model
    from gfedntm_amd.utils.config import load_config
    params = dict(load_config().training_params)
    params.update(num_epochs=1, batch_size=16, hidden_sizes=(16, 16), n_components=5)
    sc = generate_synthetic(vocab_size=80, n_topics=5, n_docs=40, n_nodes=1, frozen_topics=1,
                            nwords=(10, 20), seed=1)
    corpus = ClientCorpus(synthetic=sc, node=0)
    terms = corpus.local_terms()
    ds = build_dataset("avitm", corpus, vocabulary_dict(terms), terms)
    tm = make_topic_model("avitm", params, len(terms), torch.device("cpu"), "torch", seed=0)
    c = FederatedClient(1, tm, ds, max_iters=5)
    svc = ClientServicer(c)
    r1 = svc.getGradient(pb.ServerGetGradientRequest(iter=0), None)
    state = {k: v.clone() for k, v in tm.model.state_dict().items()}
    r2 = svc.getGradient(pb.ServerGetGradientRequest(iter=0), None)
    assert r1 is r2
    for k, v in tm.model.state_dict().items():
        assert torch.equal(v, state[k]), k            # no second local step
    hdr = pb.MessageHeader(message_type=wire.MessageType["SERVER_AGGREGATED_TENSOR_SEND"])
    msg = pb.ServerAggregatedTensorRequest(header=hdr)
    shared = {k: v for k, v in tm.model.state_dict().items() if k in set(tm.flat.shared_keys)}
    msg.nndata.modelUpdate.CopyFrom(wire.model_update_from_state(shared, 0))
    svc.sendAggregatedTensor(msg, None)
    svc.sendAggregatedTensor(msg, None)
    assert c.current_mb == 1 and c.samples_processed == int(c.plan.size[0])
