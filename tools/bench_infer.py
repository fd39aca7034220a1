"""theta-inference throughput: the HIP kernel (csrc/infer.hip, encoder once per
document, S draws in registers) vs the reference procedure on the same device
(avitm.py:470-523: S full passes of the encoder over dense [B, V] batches,
softmax of one draw each, mean) run with stock PyTorch ops.

usage: python tools/bench_infer.py [--docs 100000] [--topics 50] [--samples 20]
Prints one JSON line (docs/s of each path and the speed-up).
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import scipy.sparse as sp
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from gfedntm_amd.data.bow import DeviceCSR  # noqa: E402
from gfedntm_amd.data.synthetic import generate_synthetic, remap_to_vocabulary  # noqa: E402
from gfedntm_amd.models import AVITM  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--docs", type=int, default=100000)
    p.add_argument("--vocab", type=int, default=5000)
    p.add_argument("--topics", type=int, default=50)
    p.add_argument("--hidden", default="50,50")
    p.add_argument("--samples", type=int, default=20)
    p.add_argument("--batch", type=int, default=64, help="reference DataLoader batch")
    p.add_argument("--reps", type=int, default=5)
    p.add_argument("--no-reference", action="store_true", help="time the kernel only")
    a = p.parse_args()
    dev = torch.device("cuda")
    base = min(a.docs, 10000)                # generator is dense per node: tile a 10k-doc block
    corpus = generate_synthetic(vocab_size=a.vocab, n_topics=a.topics, n_docs=base, n_nodes=1,
                                frozen_topics=5, seed=0)
    vocab = {f"wd{i}": i for i in range(a.vocab)}
    X = remap_to_vocabulary(corpus, 0, vocab)
    X = sp.vstack([X] * (-(-a.docs // base))).tocsr()[: a.docs]
    hidden = tuple(int(h) for h in a.hidden.split(","))
    tm = AVITM(input_size=a.vocab, n_components=a.topics, hidden_sizes=hidden, batch_size=64,
               verbose=False, device=dev, backend="fused", seed=0)
    data = DeviceCSR(X, dev)
    e = tm.engine

    e.theta_infer(data, a.samples, seed=1)                   # warm-up
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for r in range(a.reps):
        th = e.theta_infer(data, a.samples, seed=r)
    torch.cuda.synchronize()
    t_kernel = (time.perf_counter() - t0) / a.reps

    if a.no_reference:
        print(json.dumps({"metric": "theta inference docs/s", "docs": data.n_docs, "K": a.topics,
                          "samples": a.samples, "kernel_docs_per_s": round(data.n_docs / t_kernel, 1),
                          "kernel_ms": round(t_kernel * 1e3, 3)}), flush=True)
        return
    # reference procedure, same device, stock ops (dense rows per batch, S passes)
    tm.model.eval()

    def reference():
        acc = None
        with torch.no_grad():
            for _ in range(a.samples):
                outs = []
                for b0 in range(0, data.n_docs, a.batch):
                    ids = torch.arange(b0, min(b0 + a.batch, data.n_docs), device=dev)
                    outs.append(tm.model.get_theta(data.dense_rows(ids)))
                t = torch.cat(outs)
                acc = t if acc is None else acc + t
        return acc / a.samples

    n_ref = min(data.n_docs, 20000)         # the reference path is slow: time a prefix
    full = data
    data = DeviceCSR(X[:n_ref], dev)
    reference()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ref = reference()
    torch.cuda.synchronize()
    t_ref = (time.perf_counter() - t0) * full.n_docs / n_ref
    out = {"metric": "theta inference docs/s", "docs": full.n_docs, "K": a.topics,
           "hidden": list(hidden), "samples": a.samples,
           "kernel_docs_per_s": round(full.n_docs / t_kernel, 1),
           "kernel_ms": round(t_kernel * 1e3, 3),
           "reference_procedure_docs_per_s": round(full.n_docs / t_ref, 1),
           "speedup": round(t_ref / t_kernel, 1),
           "mean_abs_diff_vs_reference_draws": float((th[:n_ref] - ref).abs().mean().item())}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
