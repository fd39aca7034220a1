"""Throughput of the gRPC compatibility path (BASELINE config "ProdLDA K=10, 2 clients on
synthetic BoW, CPU/gRPC reference path").

The reference's round (server.py:436-521, client.py:135-183): the server pulls every
client's shared state with getGradient, averages it sample-weighted and pushes the
aggregate back with sendAggregatedTensor; each client runs one minibatch step per round.
Here: FederationServicer + run_client (gfedntm_amd/federation/grpc_transport.py) on the
reference wire schema, server and clients in one process (threads), loopback TCP.

docs/s = clients x batch / steady-state round time (rounds after --skip).  One JSON line.
usage: python tools/bench_grpc.py [--clients 2] [--topics 10] [--iters 60] [--device cpu]
"""
import argparse
import json
import os
import socket
import sys
import tempfile
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _free_base(n):
    for base in range(43000, 60000, 37):
        ok = True
        for p in range(base, base + n + 1):
            with socket.socket() as s:
                try:
                    s.bind(("127.0.0.1", p))
                except OSError:
                    ok = False
                    break
        if ok:
            return base
    raise RuntimeError("no free ports")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=2)
    ap.add_argument("--topics", type=int, default=10)
    ap.add_argument("--vocab", type=int, default=5000)
    ap.add_argument("--docs", type=int, default=1000)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--iters", type=int, default=60)
    ap.add_argument("--skip", type=int, default=10)
    ap.add_argument("--device", default="cpu")
    ap.add_argument("--backend", default="torch")
    args = ap.parse_args()

    import numpy as np  # noqa: F401
    from gfedntm_amd.data.synthetic import generate_synthetic
    from gfedntm_amd.federation.data import ClientCorpus
    from gfedntm_amd.federation.grpc_transport import FederationServicer, run_client, serve
    from gfedntm_amd.utils.config import load_config

    params = dict(load_config().training_params)
    params.update(num_epochs=1000, batch_size=args.batch, hidden_sizes=(50, 50),
                  n_components=args.topics)
    sc = generate_synthetic(vocab_size=args.vocab, n_topics=args.topics, n_docs=args.docs,
                            n_nodes=args.clients, frozen_topics=min(5, args.topics),
                            nwords=(150, 250), seed=0)
    corpora = [ClientCorpus(synthetic=sc, node=i) for i in range(args.clients)]
    base = _free_base(args.clients)
    tmp = tempfile.mkdtemp(prefix="bench_grpc_")
    svc = FederationServicer(params, "avitm", args.clients, args.iters, client_host="127.0.0.1",
                             base_port=base, save_server=os.path.join(tmp, "server", ""),
                             wait_timeout=120)
    server = serve(svc, base)
    errors = []

    def run(i):
        try:
            run_client(corpora[i - 1], i, f"127.0.0.1:{base}", base + i, backend=args.backend,
                       device=args.device, seed=0, save_client=os.path.join(tmp, "client"),
                       timeout=120, max_iters=args.iters)
        except BaseException as e:  # pragma: no cover - reported below
            errors.append(e)

    t0 = time.perf_counter()
    ts = [threading.Thread(target=run, args=(i,)) for i in range(1, args.clients + 1)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(300)
    svc.done.wait(60)
    server.stop(0)
    if errors or svc.error is not None:
        raise SystemExit(f"gRPC federation failed: {errors or svc.error}")
    ends = svc.round_ends
    k = min(args.skip, len(ends) - 2)
    ms = 1e3 * (ends[-1] - ends[k]) / (len(ends) - 1 - k)
    # documents actually trained in the timed rounds k+1 .. len-1 (each epoch's last
    # minibatch is short: BatchPlan sizes, the clients' own plan)
    from gfedntm_amd.data.bow import BatchPlan
    docs = sum(int(BatchPlan.build(c.n_docs, args.batch, len(ends)).size[k + 1:].sum())
               for c in corpora)
    docs_s = docs / ((ends[-1] - ends[k]))
    print(json.dumps({
        "metric": f"docs/sec, ProdLDA K={args.topics} {args.clients}-client gRPC federation "
                  "(reference wire schema, loopback)",
        "value": round(docs_s, 1), "unit": "docs/s", "ms_per_round": round(ms, 3),
        "rounds": len(ends), "timed_rounds": len(ends) - 1 - k, "timed_docs": docs, "device": args.device,
        "engine": args.backend, "wall_s_total": round(time.perf_counter() - t0, 2),
        "config": {"model": f"prodLDA K={args.topics} H=(50, 50) V={len(svc.terms)}",
                   "clients": args.clients, "per_client_batch": args.batch},
        "data": "synthetic (reference LDA generator), random init",
        "baseline": {"reference_grpc_2clients_as_shipped_docs_per_s": 20.5,
                     "reference_grpc_8clients_docs_per_s": 111.0},
    }))


if __name__ == "__main__":
    main()
