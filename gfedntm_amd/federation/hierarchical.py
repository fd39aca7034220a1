"""More federated clients than ranks: hierarchical FedAvg.

The reference federates any number of clients (``--min_clients_federation``,
/root/reference/main.py:200,259; every round loops over all registered clients,
src/federation/server.py:442-484,500).  On one node the natural unit is one rank per
GPU, so with N clients on R < N ranks each rank hosts a contiguous block of clients:

  round r, rank q (clients i in block q):
    1. every local client does its local step -- fused engine: one launch per kernel
       phase for all local clients (ops/engine.py BatchedSteps, grid z = client), or one
       graph branch per client where the clients cannot be batched -- its shared state
       pre-scaled by its GLOBAL weight w_i = n_i / sum_all n;
    2. the rank folds its clients' states in client order into the first client's
       buffer (csrc/comm.hip gfk_local_fedavg, mode "first"; any number of clients);
    3. the ranks all-reduce that partial sum (the xGMI two-shot kernel: rank-order
       fold, in place for large parts; RCCL otherwise);
    4. the total is broadcast into the rank's other clients (mode "broadcast").

Steps 1-4 are one hipGraph per round when the collective is the xGMI kernel, with beta's
share (2-4) forked onto a side stream right after the decoder backward.  The sum is
fold_ranks(fold_clients_of_rank(w_i W_i)): the in-process golden with the same grouping
(``LocalFederation(..., groups=sizes)``, batched the same way) produces it bit for bit.
The round itself is federation/rank_round.py; the loop, failure detection and outputs are
the one-client-per-rank runner's (federation/runner.py run_distributed).

Control plane (gloo): the ranks agree on the client-to-rank map (every rank announces
its client ids; they must partition 1..N in rank order), the vocabulary (union of every
client's terms) and the FedAvg weights (every client's document count).
"""
from __future__ import annotations

from typing import Dict, List, Sequence

from .data import ClientCorpus


def assign_clients(n_clients: int, world: int) -> List[List[int]]:
    """Client ids 1..n_clients in contiguous blocks over ``world`` ranks (the first
    n_clients % world ranks take one more)."""
    if world < 1 or n_clients < world:
        raise ValueError(f"{n_clients} clients cannot fill {world} ranks")
    base, extra = divmod(n_clients, world)
    out, c = [], 1
    for r in range(world):
        k = base + (1 if r < extra else 0)
        out.append(list(range(c, c + k)))
        c += k
    return out


def agree_client_map(local_ids: Sequence[int], world: int, group=None) -> List[List[int]]:
    """Every rank announces its client ids; they must be contiguous blocks that partition
    1..N in rank order (the summation tree the golden reproduces)."""
    import torch.distributed as dist
    allids: List = [None] * world
    dist.all_gather_object(allids, [int(i) for i in local_ids], group=group)
    flat = [i for ids in allids for i in ids]
    if flat != list(range(1, len(flat) + 1)) or any(len(ids) == 0 for ids in allids):
        raise RuntimeError(f"client-to-rank map {allids} is not a partition of 1..{len(flat)} "
                           "into non-empty contiguous blocks in rank order")
    return allids


def run_distributed_multi(corpora: Sequence[ClientCorpus], client_ids: Sequence[int], params: Dict,
                          model_type: str = "avitm", max_iters: int = 100, **kw) -> Dict:
    """This rank's block of clients in a federation of N clients over R ranks: the same
    runner as one client per rank (:func:`~gfedntm_amd.federation.runner.run_distributed`
    with a list of corpora -- heartbeat, periodic xGMI error polls, in-place all-reduce of
    large parts, beta overlap), its rank round being federation/rank_round.py
    MultiClientRound.  Returns the rank's clients (``clients``)."""
    from .runner import run_distributed
    return run_distributed(list(corpora), params, model_type, max_iters,
                           client_ids=list(client_ids), **kw)
