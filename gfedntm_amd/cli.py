"""Command line entry (``python main.py ...``).

Reference flags (main.py:178-206): ``--id`` (0 = server / coordinator),
``--source``, ``--data_type synthetic|real``, ``--fos``,
``--min_clients_federation``, ``--model_type avitm|ctm``, ``--max_iters``.
The INI config has the reference schema (config/dft_params.cf); ``--config``
replaces the reference's hard-coded ``/workspace/config/dft_params.cf`` and
``--workdir`` is the root of the relative save / log paths.

Transports (``--backend``):
  local  all clients in this process (one GPU or CPU), exact in-process FedAvg
  rccl   one process per client over torch.distributed "nccl" (= RCCL on ROCm,
         xGMI on one node); launched by torchrun, or spawned here with --nproc
  gloo   same on CPU processes
  grpc   the reference wire protocol (federated.proto): ``--id 0`` serves, ``--id i``
         is client i
"""
from __future__ import annotations

import argparse
import datetime
import os
import socket
import sys
from typing import List, Optional

import torch


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description="gfedntm_amd: federated neural topic models on MI355X")
    # the reference README's invocation `main.py start_client --id i ...` (README.md:77; the
    # reference argparse itself has no sub-command): accepted, the role still comes from --id
    p.add_argument("command", nargs="?", default=None, choices=["start_client", "start_server"],
                   help="optional role word (reference README syntax)")
    # reference flags
    p.add_argument("--id", type=int, default=0, help="0 = server / coordinator, i >= 1 = client i")
    p.add_argument("--source", type=str, default=None, help="synthetic npz or real parquet")
    p.add_argument("--data_type", type=str, default="synthetic", choices=["synthetic", "real"])
    p.add_argument("--fos", type=str, default="computer_science",
                   help="category of the real corpus this client trains on")
    p.add_argument("--min_clients_federation", type=int, default=1)
    p.add_argument("--model_type", type=str, default="avitm", choices=["avitm", "ctm"])
    p.add_argument("--max_iters", type=int, default=25000)
    # framework flags
    p.add_argument("--config", type=str, default=None, help="INI file (reference schema)")
    p.add_argument("--workdir", type=str, default=".", help="root of relative save/log paths")
    p.add_argument("--backend", type=str, default="local",
                   choices=["local", "rccl", "gloo", "grpc"])
    p.add_argument("--nproc", type=int, default=None,
                   help="rccl/gloo: ranks to spawn when not launched by torchrun "
                        "(default min_clients_federation)")
    p.add_argument("--engine", type=str, default=None, choices=["auto", "fused", "torch"],
                   help="local-step engine (default: [amd] backend of the config)")
    p.add_argument("--device", type=str, default=None)
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--fos_list", type=str, default=None,
                   help="comma list: client i trains on category i (local / rccl / gloo)")
    p.add_argument("--log_every", type=int, default=0, help="minibatch loss line every N rounds")
    p.add_argument("--no_graph", action="store_true", help="disable hipGraph replay")
    p.add_argument("--matmul_dtype", type=str, default=None, choices=["fp32", "bf16"],
                   help="GEMM operand precision on the matrix cores (bf16: bf16 operands, fp32 "
                        "accumulation) of the ProdLDA and NeuralLDA decoders and CombinedTM's "
                        "contextual forward; parameters, Adam state and every other op stay fp32 "
                        "(default: [amd] matmul_dtype of the config)")
    p.add_argument("--agg", type=str, default="params", choices=["params", "grads"],
                   help="params: FedAvg of the shared state after every local step (reference); "
                        "grads: all-reduce of the sample-weighted gradients before one optimizer "
                        "step on every client (classic synchronous data parallelism)")
    p.add_argument("--fedavg_wire", type=str, default=None, choices=["fp32", "bf16delta"],
                   help="FedAvg transport: fp32 (reference averaging; default: [amd] fedavg_wire) "
                        "or bf16delta (opt-in: each client sends its post-step departure from "
                        "the last averaged state in bf16, summed in fp32 -- half the bytes)")
    p.add_argument("--checkpoint_dir", type=str, default=None)
    p.add_argument("--checkpoint_every", type=int, default=None)
    p.add_argument("--stop_at_num_epochs", action="store_true")
    p.add_argument("--metrics_every", type=int, default=0,
                   help="JSONL metrics window (rounds) in <logs>/metrics_<date>.jsonl; 0 = end only")
    p.add_argument("--collective_timeout", type=float, default=1800.0,
                   help="rccl/gloo: process-group timeout in seconds (failed collectives abort)")
    p.add_argument("--heartbeat_timeout", type=float, default=120.0,
                   help="rccl/gloo: seconds without a peer heartbeat before this rank aborts "
                        "(0 = off); resume with --checkpoint_dir")
    p.add_argument("--allow-pickle", dest="allow_pickle", action="store_true",
                   help="load reference synthetic npz files with object arrays (trusted files only)")
    p.add_argument("--server_address", type=str, default=None,
                   help="grpc: server host:port (default [addresses] local of the config)")
    p.add_argument("--client_host", type=str, default="127.0.0.1",
                   help="grpc: host of client i's client-server, '{id}' is replaced by i "
                        "(e.g. gfedntm-client{id})")
    p.add_argument("--server_port", type=int, default=None,
                   help="grpc: server listen port (default [federation] server_port)")
    p.add_argument("--base_port", type=int, default=None,
                   help="grpc: client i's client-server listens on base_port + i")
    p.add_argument("--generate_synthetic", type=str, default=None,
                   help="write a synthetic corpus (reference generator) to this path and use it")
    return p


def _client_fos(args, i: int) -> Optional[str]:
    if args.data_type != "real":
        return None
    if args.fos_list:
        return args.fos_list.split(",")[i - 1]
    return args.fos


def _ensure_source(args, cfg, n_nodes: int) -> str:
    if args.source:
        return args.source
    if args.data_type != "synthetic":
        raise SystemExit("--source is required for real data")
    from .data.synthetic import generate_synthetic
    path = args.generate_synthetic or os.path.join(args.workdir, "static", "datasets",
                                                   f"synthetic_{n_nodes}nodes.npz")
    if not os.path.exists(path):
        os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
        generate_synthetic(n_nodes=max(n_nodes, 1), seed=args.seed).save_counts_npz(path)
    return path


def _paths(args, cfg):
    stamp = datetime.datetime.now().strftime("%Y%m%d")
    r = lambda p: cfg.resolve(p, args.workdir)  # noqa: E731
    return stamp, r(cfg.save_client), r(cfg.save_server), r(cfg.logs_client), r(cfg.logs_server)


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def run_local(args, cfg) -> dict:
    from .federation.data import load_client_corpus
    from .federation.runner import LocalFederation
    from .utils.logging import setup_logger
    n = args.min_clients_federation
    source = _ensure_source(args, cfg, n)
    stamp, save_client, save_server, _, logs_server = _paths(args, cfg)
    logger = setup_logger("gfedntm_amd.federation", logs_server, stamp)
    corpora = [load_client_corpus(args.data_type, source, i, _client_fos(args, i), args.allow_pickle)
               for i in range(1, n + 1)]
    fed = LocalFederation(
        corpora, cfg.training_params, args.model_type, args.max_iters, device=args.device,
        metrics_path=os.path.join(logs_server, f"metrics_{stamp}.jsonl"),
        metrics_every=args.metrics_every,
        backend=args.engine or cfg.backend, grads_to_share=cfg.grads_to_share, seed=args.seed,
        save_client=save_client, save_server=save_server, logger=logger,
        graph=cfg.graph and not args.no_graph, log_every=args.log_every,
        stop_at_num_epochs=args.stop_at_num_epochs or cfg.stop_at_num_epochs,
        checkpoint_dir=args.checkpoint_dir,
        checkpoint_every=args.checkpoint_every if args.checkpoint_every is not None
        else cfg.checkpoint_every, stamp=stamp, agg=args.agg,
        fedavg_wire=args.fedavg_wire or cfg.fedavg_wire)
    return fed.run()


def _rank_main(args, cfg) -> dict:
    import torch.distributed as dist
    from .federation.data import load_client_corpus
    from .federation.runner import run_distributed
    from .utils.logging import setup_logger
    rank = dist.get_rank()
    world = dist.get_world_size()
    n_clients = max(args.min_clients_federation, world)
    source = _ensure_source(args, cfg, n_clients) if rank == 0 else None
    obj = [source]
    dist.broadcast_object_list(obj, src=0)
    source = obj[0]
    stamp, save_client, save_server, logs_client, _ = _paths(args, cfg)
    # each rank hosts a contiguous block of clients (one each when N = R; more clients
    # than ranks: hierarchical FedAvg) -- the same runner either way
    from .federation.hierarchical import assign_clients
    ids = assign_clients(n_clients, world)[rank]
    if len(ids) > 1 and args.agg != "params":
        raise SystemExit("--agg grads with more clients than ranks is not supported")
    logger = setup_logger(f"gfedntm_amd.client{ids[0]}" if len(ids) == 1 else f"gfedntm_amd.rank{rank}",
                          f"{logs_client}{ids[0]}", stamp, stdout=(rank == 0))
    corpora = [load_client_corpus(args.data_type, source, i, _client_fos(args, i), args.allow_pickle)
               for i in ids]
    return run_distributed(
        corpora[0] if len(ids) == 1 else corpora, cfg.training_params, args.model_type,
        args.max_iters, backend=args.engine or cfg.backend, grads_to_share=cfg.grads_to_share,
        seed=args.seed, save_client=save_client, save_server=save_server, logger=logger,
        graph=cfg.graph and not args.no_graph, log_every=args.log_every,
        stop_at_num_epochs=args.stop_at_num_epochs or cfg.stop_at_num_epochs,
        checkpoint_dir=args.checkpoint_dir,
        checkpoint_every=args.checkpoint_every if args.checkpoint_every is not None
        else cfg.checkpoint_every, stamp=stamp,
        metrics_path=os.path.join(f"{logs_client}{ids[0]}", f"metrics_{stamp}.jsonl"),
        metrics_every=args.metrics_every, heartbeat_timeout=args.heartbeat_timeout,
        agg_mode=args.agg, client_ids=ids, fedavg_wire=args.fedavg_wire or cfg.fedavg_wire)


def _spawned(local_rank: int, world: int, port: int, argv: List[str]):
    os.environ.update(RANK=str(local_rank), LOCAL_RANK=str(local_rank), WORLD_SIZE=str(world),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    main(argv)


def run_collective(args, cfg, argv: List[str]) -> Optional[dict]:
    import torch.distributed as dist
    if "RANK" not in os.environ:
        world = args.nproc or args.min_clients_federation
        port = _free_port()
        import torch.multiprocessing as mp
        mp.start_processes(_spawned, args=(world, port, argv), nprocs=world, start_method="spawn")
        return None
    backend = "nccl" if args.backend == "rccl" else "gloo"
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    timeout = datetime.timedelta(seconds=args.collective_timeout)
    if backend == "nccl":
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank), timeout=timeout)
    else:
        dist.init_process_group("gloo", timeout=timeout)
        if args.device is None:
            args.device = "cpu"
    try:
        return _rank_main(args, cfg)
    finally:
        dist.destroy_process_group()


def main(argv: Optional[List[str]] = None):
    argv = list(sys.argv[1:] if argv is None else argv)
    parser = build_parser()
    args = parser.parse_args(argv)
    if args.command == "start_client" and args.id == 0:
        parser.error("start_client needs --id >= 1 (0 is the server)")
    if args.command == "start_server" and args.id != 0:
        parser.error("start_server runs with --id 0")
    from .utils.config import load_config
    cfg = load_config(args.config)
    if args.matmul_dtype is not None:
        if args.matmul_dtype == "fp32":
            cfg.training_params.pop("matmul_dtype", None)
        else:
            cfg.training_params["matmul_dtype"] = args.matmul_dtype
    if args.backend == "local":
        return run_local(args, cfg)
    if args.backend in ("rccl", "gloo"):
        return run_collective(args, cfg, argv)
    if args.agg != "params":
        raise SystemExit("--agg grads needs a collective backend (local / rccl / gloo): the "
                         "reference wire protocol carries parameters, not gradients")
    if (args.fedavg_wire or cfg.fedavg_wire) != "fp32":
        raise SystemExit("--fedavg_wire bf16delta needs a collective backend (local / rccl / "
                         "gloo): the reference wire protocol carries fp32 tensors")
    from .federation import grpc_transport
    if args.id == 0:
        return grpc_transport.start_server(args, cfg)
    return grpc_transport.start_client(args, cfg)
