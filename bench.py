#!/usr/bin/env python
"""Headline benchmark: whole-node docs/s of federated ProdLDA K=50, one client per GPU.

BASELINE.json metric: "docs/sec (whole node) + NPMI, ProdLDA K=50 8-client fed on
synthetic BoW".  Config (reference config/dft_params.cf defaults + the reference
synthetic generator, src/utils/generate_synthetic.py): V=5000 generator vocabulary,
K=50 topics, hidden (50, 50), softplus, dropout 0.2, Adam(lr 2e-3, betas (0.99, 0.99)),
batch 64 per client, 1000 documents per client of 150-250 tokens, 5 frozen topics.

One *step* = one federation round exactly as the reference defines it
(federated_avitm.py:51-147 + server.py:436-521): every client does one local
minibatch step (forward, backward, Adam) and the sample-weighted average of
all shared tensors (the 20 AVITM state_dict tensors of grads_to_share) replaces
every client's copy.  On MI355X: fused HIP step (hipGraph replay) + one RCCL
all-reduce of the pre-scaled flat state over xGMI.

Weak scaling: per-GPU work (one client, batch 64) is fixed as N grows.
``value`` = N * 64 / round_time (all clients' training documents per second).
Vocabulary consensus, init broadcast and the NPMI evaluation run outside the
timed region.

Launch: ``python bench.py`` (1 GPU) or
``python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N``.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from gfedntm_amd.data.bow import BatchPlan, DeviceCSR  # noqa: E402
from gfedntm_amd.data.synthetic import (generate_synthetic, node_vocabulary_terms,  # noqa: E402
                                        remap_to_vocabulary)
from gfedntm_amd.data.vocab import union_vocabulary, vocabulary_dict  # noqa: E402
from gfedntm_amd.models import AVITM, CombinedTM, ZeroShotTM  # noqa: E402
from gfedntm_amd.parallel.aggregator import CollectiveAggregator  # noqa: E402
from gfedntm_amd.utils.config import DEFAULT_GRADS_TO_SHARE  # noqa: E402

# Reference numbers (BASELINE.md part B, measured on the unmodified reference):
# 8-client loopback gRPC federation with the built-in sleeps removed.
BASELINE_FED_DOCS_PER_S = 111.0
BASELINE_CPU_CENTRALIZED_DOCS_PER_S = 17300.0


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=2000)
    p.add_argument("--warmup", type=int, default=200)
    p.add_argument("--model", default="prodLDA", choices=["prodLDA", "LDA"])
    p.add_argument("--family", default="avitm", choices=["avitm", "ctm", "zeroshot"],
                   help="ctm = CombinedTM, zeroshot = ZeroShotTM, with --contextual-size "
                        "synthetic embeddings")
    p.add_argument("--contextual-size", type=int, default=768)
    p.add_argument("--vocab", type=int, default=5000)
    p.add_argument("--topics", type=int, default=50)
    p.add_argument("--hidden", default="50,50")
    p.add_argument("--batch", type=int, default=64)
    p.add_argument("--docs", type=int, default=1000)
    p.add_argument("--backend", default="fused", choices=["fused", "torch"])
    p.add_argument("--no-graph", action="store_true")
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--no-npmi", action="store_true")
    p.add_argument("--solver", default="adam",
                   choices=["adam", "sgd", "adagrad", "adadelta", "rmsprop"],
                   help="optimizer (reference default adam; the others run in gradient mode)")
    return p.parse_args()


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # GFEDNTM_REHEARSE_1GPU=1: rehearse the multi-rank path on a one-GPU box -- every
    # rank on cuda:0, gloo process group (timings are meaningless, the code path and
    # the xGMI all-reduce protocol are the real ones)
    rehearse = os.environ.get("GFEDNTM_REHEARSE_1GPU") == "1"
    if rehearse:
        local_rank = 0
    if world > 1:
        torch.cuda.set_device(local_rank)
        if rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    device = torch.device("cuda", local_rank)
    n_clients = world

    # ---- data: reference synthetic generator, one node per client ----
    corpus = generate_synthetic(vocab_size=args.vocab, n_topics=args.topics, n_docs=args.docs,
                                n_nodes=max(n_clients, 1), frozen_topics=5, seed=args.seed)
    # ---- stage 1: vocabulary consensus (sorted union of local vocabularies) ----
    local_terms = node_vocabulary_terms(corpus, rank)
    if world > 1:
        gathered = [None] * world
        dist.all_gather_object(gathered, local_terms)
    else:
        gathered = [local_terms]
    terms = union_vocabulary(gathered)
    vocab = vocabulary_dict(terms)
    X = remap_to_vocabulary(corpus, rank, vocab)

    hidden = tuple(int(h) for h in args.hidden.split(","))
    torch.manual_seed(args.seed)
    kw = dict(input_size=len(terms), n_components=args.topics, model_type=args.model,
              hidden_sizes=hidden, batch_size=args.batch, verbose=False, backend=args.backend,
              device=device, shared_keys=DEFAULT_GRADS_TO_SHARE, seed=args.seed,
              solver=args.solver)
    ctx = None
    if args.family in ("ctm", "zeroshot"):
        # SBERT is not available offline: per-document embeddings are synthetic
        # (a fixed random projection of the document's topic mixture plus noise)
        rng = np.random.default_rng(args.seed + 17 * rank)
        proj = np.random.default_rng(args.seed).standard_normal(
            (args.topics, args.contextual_size)).astype(np.float32)
        ctx = (np.asarray(corpus.doc_topics[rank], dtype=np.float32) @ proj
               + 0.1 * rng.standard_normal((X.shape[0], args.contextual_size)).astype(np.float32))
        cls = CombinedTM if args.family == "ctm" else ZeroShotTM
        tm = cls(contextual_size=args.contextual_size, **kw)
    else:
        tm = AVITM(**kw)
    eng = tm.engine
    agg, comm = None, None
    if world > 1:
        dist.broadcast(tm.flat.buffer, src=0)        # identical W0 on every client
        agg = CollectiveAggregator(method="rccl")
        w = agg.weights(X.shape[0], device)
        if args.backend == "fused":
            eng.set_fedavg_scale(w[rank])
            # the all-reduce becomes part of the step (custom xGMI kernel captured in the
            # step graph, beta's share overlapped with the encoder backward) or follows
            # it (RCCL) -- see FusedEngine.attach_fedavg
            comm = eng.attach_fedavg()
        else:
            comm = agg.prepare(tm.flat.shared)
    data = DeviceCSR(X, device, contextual=ctx)
    n_steps = args.warmup + args.steps
    plan = BatchPlan.build(data.n_docs, args.batch, n_steps, seed=args.seed + rank)
    eng.bind_data(data, plan)
    if args.backend == "fused" and not args.no_graph:
        eng.enable_graph(True)
        eng.warm_graph()
    if world > 1:                 # ranks enter the first (collective) step together
        torch.cuda.synchronize()
        dist.barrier()

    shared = tm.flat.shared

    def round_(s):
        eng.step(s)
        if agg is not None and args.backend != "fused":
            shared.mul_(w[rank])
            agg.allreduce_(shared)

    for s in range(args.warmup):
        round_(s)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for s in range(args.warmup, n_steps):
        round_(s)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    comm_error = eng.fedavg_error() if args.backend == "fused" else 0
    if comm_error:                              # a timed-out wait invalidates the run
        raise RuntimeError(f"xGMI all-reduce reported error {comm_error}")
    ms = dt / args.steps * 1e3
    docs_per_s = n_clients * args.batch * args.steps / dt
    losses = eng.loss_hist.detach().cpu().numpy()

    npmi = None
    if rank == 0 and not args.no_npmi:
        from gfedntm_amd.eval.metrics import npmi_coherence
        from gfedntm_amd.data.synthetic import remap_to_vocabulary as remap
        import scipy.sparse as sp
        ref_corpus = sp.vstack([remap(corpus, i, vocab) for i in range(max(n_clients, 1))])
        topics_idx = torch.topk(tm.model.beta.detach(), 10, dim=1).indices.cpu().numpy()
        npmi = float(npmi_coherence(topics_idx, ref_corpus, device=device))

    # round latency split (BASELINE: compute / all-reduce / host): the same number of
    # steps again with the collective detached, after the timed region
    split = None
    if world > 1 and args.backend == "fused" and eng._comm is not None:
        saved_comm = eng._comm
        eng._comm = None
        eng._invalidate_graph()
        k2 = max(1, min(args.steps, 500))
        for s in range(n_steps, n_steps + min(args.warmup, 50)):
            eng.step(s % n_steps)
        torch.cuda.synchronize()
        dist.barrier()
        t1 = time.perf_counter()
        for s in range(k2):
            eng.step(s % n_steps)
        torch.cuda.synchronize()
        tc = torch.tensor([(time.perf_counter() - t1) / k2 * 1e3], dtype=torch.float64,
                          device=device)
        dist.all_reduce(tc, op=dist.ReduceOp.MAX)
        eng._comm = saved_comm
        split = {"compute_ms": round(float(tc.item()), 5)}
    if split is not None:
        split["allreduce_exposed_ms"] = round(max(ms - split["compute_ms"], 0.0), 5)

    if rank == 0:
        out = {
            "metric": "docs/sec (whole node) + NPMI, ProdLDA K=50 8-client fed on synthetic BoW",
            "value": round(docs_per_s, 1),
            "unit": "docs/s",
            "n_gpus": n_clients,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 5),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(docs_per_s / BASELINE_FED_DOCS_PER_S, 2),
            "dtype": "fp32",
            "data": "synthetic (reference LDA generator: V=5000, K=50, 1000 docs/client, "
                    "150-250 tokens, 5 frozen topics), random init",
            "config": {"model": ((f"CombinedTM-{args.model} C={args.contextual_size}"
                                  if args.family == "ctm" else
                                  f"ZeroShotTM-{args.model} C={args.contextual_size}")
                                 if args.family in ("ctm", "zeroshot") else args.model)
                                + f" K={args.topics} H={hidden} V={len(terms)}",
                       "global_batch": args.batch * n_clients, "seq_len": None,
                       "per_client_batch": args.batch, "clients": n_clients,
                       "parallelism": f"fedavg-dp{n_clients}",
                       "backend": args.backend + ("" if args.no_graph else "+hipgraph"),
                       "solver": args.solver,
                       "aggregation": "per-minibatch sample-weighted FedAvg of 20 shared tensors"
                                      + (f" ({comm} all-reduce)" if world > 1 else "")},
            "npmi": None if npmi is None else round(npmi, 4),
            "round_split_ms": split if split is not None else {"compute_ms": round(ms, 5),
                                                               "allreduce_exposed_ms": 0.0},
            "final_loss": float(np.mean(losses[-20:])),
            "baseline": {"fed_grpc_8clients_docs_per_s": BASELINE_FED_DOCS_PER_S,
                         "cpu_centralized_docs_per_s": BASELINE_CPU_CENTRALIZED_DOCS_PER_S},
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
