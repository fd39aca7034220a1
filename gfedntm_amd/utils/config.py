"""INI configuration for gfedntm_amd.

Accepts the reference's `config/dft_params.cf` schema unchanged
(reference: config/dft_params.cf:1-55) and reproduces the typing rules of
`read_config_experiments` (reference: src/utils/auxiliary_functions.py:387-438):
all sections are flattened into one dict, and values are typed by key name.
Two reference quirks are kept on purpose because the federation forwards this
dict verbatim to every client: ``labels`` is always ``""`` and
``topic_prior_variance`` is always ``None`` (-> 1 - 1/K inside the model).

On top of that this module adds a typed view (:class:`FedConfig`) with the
sections the reference reads through raw ``configparser.get`` calls in
main.py:213-254 (addresses, grpc, federation, save_dir) plus an ``[amd]``
section for MI355X-only knobs.
"""
from __future__ import annotations

import configparser
import dataclasses
import os
from typing import Any, Dict, List, Optional

_INT_KEYS = {
    "n_components", "num_iterations", "batch_size", "num_threads",
    "optimize_interval", "num_epochs", "num_samples",
    "num_data_loader_workers", "contextual_size",
}
_FLOAT_KEYS = {
    "thetas_thr", "doc_topic_thr", "alpha", "dropout", "lr", "momentum",
    "topic_prior_mean",
}
_BOOL_KEYS = {"learn_priors", "reduce_on_plateau", "verbose"}

DEFAULT_CONFIG = os.path.join(
    os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
    "config", "dft_params.cf")

# Reference default list of shared tensors (config/dft_params.cf:50).
DEFAULT_GRADS_TO_SHARE: List[str] = [
    "prior_mean", "prior_variance", "beta",
    "inf_net.f_mu_batchnorm.num_batches_tracked",
    "inf_net.f_sigma_batchnorm.num_batches_tracked",
    "beta_batchnorm.num_batches_tracked",
    "inf_net.input_layer.weight", "inf_net.input_layer.bias",
    "inf_net.hiddens.l_0.0.weight", "inf_net.hiddens.l_0.0.bias",
    "inf_net.f_mu.weight", "inf_net.f_mu.bias",
    "inf_net.f_mu_batchnorm.running_mean", "inf_net.f_mu_batchnorm.running_var",
    "inf_net.f_sigma.weight", "inf_net.f_sigma.bias",
    "inf_net.f_sigma_batchnorm.running_mean",
    "inf_net.f_sigma_batchnorm.running_var",
    "beta_batchnorm.running_mean", "beta_batchnorm.running_var",
    "inf_net.adapt_bert.weight", "inf_net.adapt_bert.bias",
]


def _parse_hidden(value: str):
    value = value.strip()
    if value.startswith("(") and value.endswith(")"):
        value = value[1:-1]
    return tuple(int(v) for v in value.split(",") if v.strip())


def type_value(option: str, value: str) -> Any:
    """Types one INI value exactly like the reference's key-name lists."""
    if option in _INT_KEYS:
        return int(value)
    if option in _FLOAT_KEYS:
        return float(value)
    if option == "labels":
        return ""
    if option == "topic_prior_variance":
        return None
    if option in _BOOL_KEYS:
        return value == "True"
    if option == "hidden_sizes":
        return _parse_hidden(value)
    return value


def read_config_experiments(file_path: str, skip: Optional[List[str]] = None) -> Dict[str, Any]:
    """Flattened, typed config dict (reference auxiliary_functions.py:387-438)."""
    skip = skip or []
    cp = configparser.ConfigParser()
    if not cp.read(file_path):
        raise FileNotFoundError(file_path)
    out: Dict[str, Any] = {}
    for section in cp.sections():
        if section in skip:
            continue
        for option in cp.options(section):
            out[option] = type_value(option, cp.get(section, option))
    return out


@dataclasses.dataclass
class FedConfig:
    """Typed view of the whole INI file."""

    training_params: Dict[str, Any]
    address: str = "gfedntm-server:50051"
    local_address: str = "localhost:50051"
    base_port: int = 50051
    grpc_max_message_length: int = 262144000
    grpc_max_inbound_message_size: int = 262144000
    grpc_max_inbound_metadata_size: int = 262144000
    grpc_keepalive_time_ms: int = 10000
    grpc_keepalive_timeout_ms: int = 5000
    grpc_keepalive_permit_without_calls: bool = True
    grpc_max_ping_strikes: int = 0
    time_termination: int = 604800
    server_port: int = 50051
    client_sleep_time: int = 604800
    grads_to_share: List[str] = dataclasses.field(
        default_factory=lambda: list(DEFAULT_GRADS_TO_SHARE))
    save_client: str = "static/output_models/client"
    save_server: str = "static/output_models/server"
    logs_client: str = "static/logs/client"
    logs_server: str = "static/logs/server"
    backend: str = "fused"
    graph: bool = True
    aggregate: str = "params"
    checkpoint_every: int = 0
    stop_at_num_epochs: bool = False
    # FedAvg wire: "fp32" (the reference's averaging) | "bf16delta" (opt-in, half the bytes)
    fedavg_wire: str = "fp32"

    def grpc_client_options(self):
        """Channel options used by a process dialing out (reference main.py:219-231)."""
        m = self.grpc_max_message_length
        return [
            ("grpc.max_message_length", m),
            ("grpc.max_send_message_length", m),
            ("grpc.max_receive_message_length", m),
            ("grpc.max_inbound_message_size", self.grpc_max_inbound_message_size),
            ("grpc.max_inbound_metadata_size", self.grpc_max_inbound_metadata_size),
            ("grpc.max_metadata_size", self.grpc_max_inbound_metadata_size),
        ]

    def grpc_server_options(self):
        """Options of a process serving RPCs (reference main.py:234-242)."""
        m = self.grpc_max_message_length
        return [
            ("grpc.max_send_message_length", m),
            ("grpc.max_receive_message_length", m),
            ("grpc.keepalive_time_ms", self.grpc_keepalive_time_ms),
            ("grpc.keepalive_timeout_ms", self.grpc_keepalive_timeout_ms),
            ("grpc.keepalive_permit_without_calls",
             bool(self.grpc_keepalive_permit_without_calls)),
            ("grpc.http2.max_ping_strikes", self.grpc_max_ping_strikes),
        ]

    def resolve(self, path: str, workdir: str) -> str:
        return path if os.path.isabs(path) else os.path.join(workdir, path)


def load_config(file_path: Optional[str] = None) -> FedConfig:
    """Reads an INI file (default: repo config/dft_params.cf) into a FedConfig."""
    file_path = file_path or DEFAULT_CONFIG
    params = read_config_experiments(file_path, skip=["amd"])
    cp = configparser.ConfigParser()
    cp.read(file_path)

    def get(section, key, default, cast=str):
        if cp.has_option(section, key):
            raw = cp.get(section, key)
            if cast is bool:
                return raw.strip() == "True"
            return cast(raw)
        return default

    cfg = FedConfig(training_params=params)
    cfg.address = get("addresses", "docker", cfg.address)
    cfg.local_address = get("addresses", "local", cfg.local_address)
    cfg.base_port = get("addresses", "base_port", cfg.base_port, int)
    cfg.grpc_max_message_length = get("grpc", "max_message_length", cfg.grpc_max_message_length, int)
    cfg.grpc_max_inbound_message_size = get("grpc", "max_inbound_message_size",
                                            cfg.grpc_max_inbound_message_size, int)
    cfg.grpc_max_inbound_metadata_size = get("grpc", "max_inbound_metadata_size",
                                             cfg.grpc_max_inbound_metadata_size, int)
    cfg.grpc_keepalive_time_ms = get("grpc", "keepalive_time_ms", cfg.grpc_keepalive_time_ms, int)
    cfg.grpc_keepalive_timeout_ms = get("grpc", "keepalive_timeout_ms",
                                        cfg.grpc_keepalive_timeout_ms, int)
    cfg.grpc_keepalive_permit_without_calls = get(
        "grpc", "keepalive_permit_without_calls", cfg.grpc_keepalive_permit_without_calls, bool)
    cfg.grpc_max_ping_strikes = get("grpc", "max_ping_strikes", cfg.grpc_max_ping_strikes, int)
    cfg.time_termination = get("federation", "time_termination", cfg.time_termination, int)
    cfg.server_port = get("federation", "server_port", cfg.server_port, int)
    cfg.client_sleep_time = get("federation", "client_sleep_time", cfg.client_sleep_time, int)
    if cp.has_option("federation", "grads_to_share"):
        cfg.grads_to_share = [k.strip() for k in cp.get("federation", "grads_to_share").split(",")
                              if k.strip()]
    cfg.save_client = get("save_dir", "save_client", cfg.save_client)
    cfg.save_server = get("save_dir", "save_server", cfg.save_server)
    cfg.logs_client = get("save_dir", "logs_client", cfg.logs_client)
    cfg.logs_server = get("save_dir", "logs_server", cfg.logs_server)
    cfg.backend = get("amd", "backend", cfg.backend)
    cfg.graph = get("amd", "graph", cfg.graph, bool)
    cfg.aggregate = get("amd", "aggregate", cfg.aggregate)
    cfg.checkpoint_every = get("amd", "checkpoint_every", cfg.checkpoint_every, int)
    cfg.stop_at_num_epochs = get("amd", "stop_at_num_epochs", cfg.stop_at_num_epochs, bool)
    cfg.fedavg_wire = get("amd", "fedavg_wire", cfg.fedavg_wire)
    if cfg.fedavg_wire not in ("fp32", "bf16delta"):
        raise ValueError(f"[amd] fedavg_wire must be fp32 or bf16delta, got {cfg.fedavg_wire!r}")
    mm = get("amd", "matmul_dtype", "fp32")
    if mm != "fp32":
        cfg.training_params["matmul_dtype"] = mm
    return cfg


def model_kwargs_from_params(params: Dict[str, Any]) -> Dict[str, Any]:
    """Subset of the flattened dict that the topic models consume."""
    keys = ["n_components", "model_type", "hidden_sizes", "activation", "dropout",
            "learn_priors", "batch_size", "lr", "momentum", "solver", "num_epochs",
            "reduce_on_plateau", "topic_prior_mean", "topic_prior_variance",
            "num_samples", "num_data_loader_workers", "verbose", "matmul_dtype"]
    return {k: params[k] for k in keys if k in params}
