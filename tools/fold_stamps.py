"""Diagnostic: phase stamps (s_memtime, workgroup 0) of the in-epilogue FedAvg backward
(csrc/prodlda.hip gfk_bwd_fold_k) in the 8-client headline round.

  python tools/fold_stamps.py --build-only     (host: builds build/stamps/libgfedntm_kernels.so)
  GFEDNTM_KERNELS_SO=build/stamps/libgfedntm_kernels.so python tools/fold_stamps.py   (GPU)
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--build-only", action="store_true")
    p.add_argument("--clients", type=int, default=8)
    a = p.parse_args()
    if a.build_only:
        from tools.stamps import build
        print(build())
        return
    import torch
    from gfedntm_amd.data.synthetic import generate_synthetic
    from gfedntm_amd.federation.data import ClientCorpus
    from gfedntm_amd.federation.runner import LocalFederation
    from gfedntm_amd.utils.config import load_config
    M = a.clients
    sc = generate_synthetic(vocab_size=5000, n_topics=50, n_docs=1000 * M, n_nodes=M,
                            frozen_topics=5, nwords=(150, 250), seed=0)
    corpora = [ClientCorpus(synthetic=sc, node=i) for i in range(M)]
    prm = dict(load_config().training_params)
    prm.update(num_epochs=100, batch_size=64, hidden_sizes=(50, 50), n_components=50)
    fed = LocalFederation(corpora, prm, max_iters=30, device="cuda", backend="fused", seed=1,
                          round_batched=True)
    dbg = torch.zeros(4096, dtype=torch.int64, device="cuda")
    for c in fed.clients:
        c.tm.engine._m.dbg = dbg.data_ptr()
    fed.run()
    torch.cuda.synchronize()
    d = dbg.cpu().numpy()
    print("fold plan:", fed.fold_plan)
    t0 = d[98]
    print("start->prologue issued", d[100] - t0, " prologue staged", d[101] - t0, " end", d[99] - t0)
    w0 = d[298]
    print("win: start->prologue", d[300] - w0, d[301] - w0, " end", d[299] - w0)
    for c in range(M):
        s = [d[302 + 8 * c + i] for i in range(7)]
        print(f"win client {c}: top {s[0] - w0:6d} | issue {s[1] - s[0]:5d} mfma {s[2] - s[1]:5d} "
              f"barrier {s[3] - s[2]:5d} adam {s[4] - s[3]:5d} barrier {s[5] - s[4]:5d} stage {s[6] - s[5]:5d}")
    for c in range(M):
        s = [d[102 + 8 * c + i] for i in range(7)]
        print(f"client {c}: top {s[0] - t0:6d} | issue+sparse {s[1] - s[0]:5d} barrier {s[2] - s[1]:5d} "
              f"dense {s[3] - s[2]:5d} mfma {s[4] - s[3]:5d} adam {s[5] - s[4]:5d} stage {s[6] - s[5]:5d}")


if __name__ == "__main__":
    main()
