"""Round-level checkpoints for federated training (the reference has none).

One file per client: ``{dir}/client{id}_round{r}.pt`` holding the model state_dict
(parameters + batch-norm buffers), the optimizer state (torch.optim format, also
for the fused engine), the loss history, the round index and the client's
bookkeeping.  Everything is tensors / primitives, so it loads with
``torch.load(weights_only=True)``.  The batch plan is a pure function of
(seed, n_docs, batch, max_iters), so it is rebuilt, not stored; the fused
engine's Philox draws are keyed by (seed, step) and resume exactly.
"""
from __future__ import annotations

import glob
import os
import re
from typing import Optional

import torch

_BOOK = ("current_mb", "current_epoch", "samples_processed", "train_loss", "epoch_first_step",
         "results_saved")


def checkpoint_path(ckpt_dir: str, client_id: int, round_: int) -> str:
    return os.path.join(ckpt_dir, f"client{client_id}_round{round_}.pt")


def save_client_checkpoint(ckpt_dir: str, client, round_: int) -> str:
    os.makedirs(ckpt_dir, exist_ok=True)
    if hasattr(client, "flush"):      # pending epoch summaries update the bookkeeping
        client.flush()
    tm = client.tm
    eng = tm.engine
    state = {
        "round": int(round_),
        "state_dict": {k: v.detach().cpu() for k, v in tm.model.state_dict().items()},
        "optimizer": eng.optimizer_state_dict(),
        "loss_hist": eng.loss_hist[:round_].detach().cpu(),
        "book": {k: getattr(client, k) for k in _BOOK},
        "best_loss_train": float(tm.best_loss_train),
        "seed": int(getattr(eng, "seed", 0)),
        # the global RNG (anything not on an engine-owned stream)
        "rng_cpu": torch.get_rng_state(),
        "rng_cuda": (torch.cuda.get_rng_state(eng.device) if eng.device.type == "cuda"
                     else torch.zeros(0, dtype=torch.uint8)),
    }
    if getattr(eng, "rng_state", None) is not None and eng.rng_state() is not None:
        # the PyTorch engine's own per-client noise stream (cpu, device)
        cpu_st, dev_st = eng.rng_state()
        state["rng_engine_cpu"] = cpu_st
        state["rng_engine_dev"] = dev_st if dev_st is not None else torch.zeros(0, dtype=torch.uint8)
    if hasattr(eng, "adam_pow"):
        # the fused kernels advance beta^t on device by repeated fp64 products;
        # recomputing beta ** t on resume could differ in the last bit, so the device
        # values travel verbatim (bitwise-exact resume)
        state["adam_pow"] = eng.adam_pow.detach().cpu()
        state["adam_coef"] = eng.adam_coef.detach().cpu()
    path = checkpoint_path(ckpt_dir, client.id, round_)
    tmp = path + ".tmp"
    torch.save(state, tmp)
    os.replace(tmp, path)
    return path


def latest_round(ckpt_dir: str, client_id: int) -> Optional[int]:
    rounds = []
    for p in glob.glob(os.path.join(ckpt_dir, f"client{client_id}_round*.pt")):
        m = re.search(r"_round(\d+)\.pt$", p)
        if m:
            rounds.append(int(m.group(1)))
    return max(rounds) if rounds else None


def load_client_checkpoint(ckpt_dir: str, client, round_: Optional[int] = None) -> int:
    """Restores a client in place; returns the round to continue from."""
    round_ = latest_round(ckpt_dir, client.id) if round_ is None else round_
    if round_ is None:
        return 0
    st = torch.load(checkpoint_path(ckpt_dir, client.id, round_), map_location="cpu",
                    weights_only=True)
    tm = client.tm
    eng = tm.engine
    tm.model.load_state_dict(st["state_dict"])
    eng.load_optimizer_state_dict(st["optimizer"])
    eng.loss_hist[: st["round"]].copy_(st["loss_hist"].to(eng.loss_hist.device))
    for k, v in st["book"].items():
        setattr(client, k, v)
    tm.best_loss_train = st["best_loss_train"]
    torch.set_rng_state(st["rng_cpu"])
    if eng.device.type == "cuda" and st["rng_cuda"].numel():
        torch.cuda.set_rng_state(st["rng_cuda"], eng.device)
    if "rng_engine_cpu" in st and hasattr(eng, "set_rng_state"):
        dev_st = st["rng_engine_dev"]
        eng.set_rng_state((st["rng_engine_cpu"], dev_st if dev_st.numel() else None))
    if hasattr(eng, "adam_pow") and "adam_pow" in st:
        eng.adam_pow.copy_(st["adam_pow"].to(eng.adam_pow.device))
        eng.adam_coef.copy_(st["adam_coef"].to(eng.adam_coef.device))
    if hasattr(eng, "seed") and hasattr(eng, "_m"):
        eng.seed = st["seed"]
        eng._m.seed = st["seed"]
        eng._invalidate_graph()
    return int(st["round"])
