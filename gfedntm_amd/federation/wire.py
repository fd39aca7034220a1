"""The reference wire schema (src/protos/federated.proto) and its codecs.

``grpc_tools``/``protoc`` are not available on this image, so the schema is
assembled directly as a ``FileDescriptorProto`` -- same package (``federated``),
message names, field names, numbers, types, labels and oneofs as the reference
proto, hence byte-compatible on the wire with the reference clients / server.

Codecs (reference src/utils/auxiliary_functions.py:24-385):
  * tensors travel as ``Tensor{shape (Dim size[, name]), dtype string, raw bytes}``
    with dtype in {float32, float64, int64};
  * a state_dict maps to the fixed 24-field ``ModelUpdate`` by replacing '.' with
    '_', except the first hidden layer (fields ``inf_net_hiddens_l00_weight`` and
    ``inf_net_hiddens_l_00_bias``); the fixed schema therefore carries at most one
    hidden-to-hidden layer (hidden_sizes of length <= 2) and no CTM label head;
  * ``AdamUpdate`` carries torch's Adam ``state_dict`` (per-parameter step /
    exp_avg / exp_avg_sq, one param group);
  * ``Dictionary`` carries the vocabulary (term -> int32) and the typed model
    parameters (str / int32 / float32 / int tuple / bool).
"""
from __future__ import annotations

from typing import Any, Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch
from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

PACKAGE = "federated"
_F = descriptor_pb2.FieldDescriptorProto
_TYPES = {"int64": _F.TYPE_INT64, "uint32": _F.TYPE_UINT32, "int32": _F.TYPE_INT32,
          "string": _F.TYPE_STRING, "bytes": _F.TYPE_BYTES, "float": _F.TYPE_FLOAT,
          "bool": _F.TYPE_BOOL}

# message -> [(field, number, type, label, oneof)], type "M:<Name>" / "E:<Name>" for
# message / enum references (relative to the package), label in {"", "repeated",
# "optional"} (proto3 explicit presence), oneof = name of the containing oneof.
_MODEL_UPDATE_FIELDS = [
    "prior_mean", "prior_variance", "beta", "topic_word_matrix", "inf_net_input_layer_weight",
    "inf_net_input_layer_bias", "inf_net_hiddens_l00_weight", "inf_net_hiddens_l_00_bias",
    "inf_net_f_mu_weight", "inf_net_f_mu_bias", "inf_net_f_mu_batchnorm_running_mean",
    "inf_net_f_mu_batchnorm_running_var", "inf_net_f_mu_batchnorm_num_batches_tracked",
    "inf_net_f_sigma_weight", "inf_net_f_sigma_bias", "inf_net_f_sigma_batchnorm_running_mean",
    "inf_net_f_sigma_batchnorm_running_var", "inf_net_f_sigma_batchnorm_num_batches_tracked",
    "beta_batchnorm_running_mean", "beta_batchnorm_running_var",
    "beta_batchnorm_num_batches_tracked", "best_components", "inf_net_adapt_bert_weight",
    "inf_net_adapt_bert_bias",
]

_SCHEMA: List[Tuple[str, list]] = [
    ("Empty", []),
    ("TensorShape.Dim", [("size", 1, "int64", "", None), ("name", 2, "string", "optional", None)]),
    ("TensorShape", [("dim", 2, "M:TensorShape.Dim", "repeated", None)]),
    ("Tensor", [("tensor_shape", 1, "M:TensorShape", "", None), ("dtype", 2, "string", "", None),
                ("tensor_content", 3, "bytes", "", None)]),
    ("Update", [("tensor_name", 1, "string", "", None), ("tensor", 2, "M:Tensor", "", None)]),
    ("MessageAdditionalData", [("current_mb", 1, "uint32", "", None),
                               ("current_epoch", 2, "uint32", "", None),
                               ("num_max_epochs", 3, "uint32", "", None),
                               ("id_machine", 4, "uint32", "", None)]),
    ("MessageHeader", [("id_request", 1, "string", "optional", None),
                       ("id_response", 2, "string", "optional", None),
                       ("id_to_request", 3, "string", "optional", None),
                       ("message_type", 4, "E:MessageType", "", None)]),
    ("ClientTensorRequest", [("header", 1, "M:MessageHeader", "", None),
                             ("metadata", 2, "M:MessageAdditionalData", "", None),
                             ("updates", 3, "M:Update", "repeated", None)]),
    ("ServerAggregatedTensorRequest", [("header", 1, "M:MessageHeader", "", None),
                                       ("metadata", 2, "M:MessageAdditionalData", "", None),
                                       ("data", 3, "M:Update", "", "oneof_values"),
                                       ("nndata", 4, "M:NNUpdate", "", "oneof_values")]),
    ("ClientReceivedResponse", [("header", 1, "M:MessageHeader", "", None),
                                ("metadata", 2, "M:MessageAdditionalData", "", None)]),
    ("ServerReceivedResponse", [("header", 1, "M:MessageHeader", "", None),
                                ("metadata", 2, "M:MessageAdditionalData", "", None)]),
    ("Chunk", [("buffer", 1, "bytes", "", None)]),
    ("Request", [("name", 1, "string", "", None)]),
    ("Reply", [("length", 1, "int32", "", None)]),
    ("Tuple.Valuet", [("svalue", 1, "string", "", "oneof_values"),
                      ("ivalue", 2, "int32", "", "oneof_values"),
                      ("fvalue", 3, "float", "", "oneof_values")]),
    ("Tuple", [("values", 1, "M:Tuple.Valuet", "repeated", None)]),
    ("Dictionary.Pair.Value", [("svalue", 1, "string", "", "oneof_values"),
                               ("ivalue", 2, "int32", "", "oneof_values"),
                               ("fvalue", 3, "float", "", "oneof_values"),
                               ("tvalue", 4, "M:Tuple", "", "oneof_values"),
                               ("bvalue", 5, "bool", "", "oneof_values")]),
    ("Dictionary.Pair", [("key", 1, "string", "", None),
                         ("value", 2, "M:Dictionary.Pair.Value", "", None)]),
    ("Dictionary", [("pairs", 1, "M:Dictionary.Pair", "repeated", None)]),
    ("DictRequest", [("vocab", 1, "M:Dictionary", "", None), ("client_id", 2, "int32", "", None),
                     ("nr_samples", 3, "int32", "", None)]),
    ("FeatureUnion", [("dic", 1, "M:Dictionary", "repeated", None),
                      ("initialNN", 2, "M:NNUpdate", "", None),
                      ("model_params", 3, "M:Dictionary", "", None),
                      ("model_type", 4, "string", "", None)]),
    ("ModelUpdate", [(f, i + 1, "M:Tensor", "", None) for i, f in enumerate(_MODEL_UPDATE_FIELDS)]
     + [("current_epoch", 25, "int32", "", None)]),
    ("AdamUpdate.State.ContentState", [("state_id", 1, "int64", "", None),
                                       ("step", 2, "M:Tensor", "", None),
                                       ("exp_avg", 3, "M:Tensor", "", None),
                                       ("exp_avg_sq", 4, "M:Tensor", "", None)]),
    ("AdamUpdate.State", [("contentState", 2, "M:AdamUpdate.State.ContentState", "repeated", None)]),
    ("AdamUpdate.ParamGroups.Betas", [("beta1", 1, "float", "", None), ("beta2", 2, "float", "", None)]),
    ("AdamUpdate.ParamGroups", [("lr", 1, "float", "", None),
                                ("betas", 2, "M:AdamUpdate.ParamGroups.Betas", "", None),
                                ("eps", 3, "float", "", None), ("weight_decay", 4, "float", "", None),
                                ("amsgrad", 5, "bool", "", None), ("params", 6, "int32", "repeated", None)]),
    ("AdamUpdate", [("state", 1, "M:AdamUpdate.State", "", None),
                    ("paramGroups", 2, "M:AdamUpdate.ParamGroups", "", None)]),
    ("OptUpdate", [("adamUpdate", 1, "M:AdamUpdate", "", "oneof_values")]),
    ("NNUpdate", [("modelUpdate", 1, "M:ModelUpdate", "", None), ("optUpdate", 2, "M:OptUpdate", "", None)]),
    ("ServerGetGradientRequest", [("iter", 1, "int64", "", None)]),
]

MESSAGE_TYPES = ["CLIENT_TENSOR_SEND", "CLIENT_CONFIRM_RECEIVED", "CLIENT_READY_FOR_TRAINING",
                 "SERVER_AGGREGATED_TENSOR_SEND", "SERVER_CONFIRM_RECEIVED",
                 "SERVER_STOP_TRAINING_REQUEST"]

# service -> method -> (request, response)
SERVICES = {
    "Federation": {
        "sendAggregatedTensor": ("Empty", "ServerAggregatedTensorRequest"),
        "sendLocalDic": ("DictRequest", "Reply"),
        "sendGlobalDicAndInitialNN": ("Empty", "FeatureUnion"),
        "trainFederatedModel": ("ClientTensorRequest", "Empty"),
    },
    "FederationServer": {
        "getGradient": ("ServerGetGradientRequest", "ClientTensorRequest"),
        "sendAggregatedTensor": ("ServerAggregatedTensorRequest", "ClientReceivedResponse"),
    },
}


def _build_file() -> descriptor_pb2.FileDescriptorProto:
    fd = descriptor_pb2.FileDescriptorProto(name="federated.proto", package=PACKAGE, syntax="proto3")
    en = fd.enum_type.add(name="MessageType")
    for i, n in enumerate(MESSAGE_TYPES):
        en.value.add(name=n, number=i)
    protos: Dict[str, descriptor_pb2.DescriptorProto] = {}
    for path, fields in sorted(_SCHEMA, key=lambda e: e[0].count(".")):
        parts = path.split(".")
        parent = None if len(parts) == 1 else protos[".".join(parts[:-1])]
        msg = (fd.message_type if parent is None else parent.nested_type).add(name=parts[-1])
        protos[path] = msg
        oneofs: Dict[str, int] = {}
        for name, number, typ, label, oneof in fields:
            f = msg.field.add(name=name, number=number, json_name=name)
            f.label = _F.LABEL_REPEATED if label == "repeated" else _F.LABEL_OPTIONAL
            if typ.startswith("M:"):
                f.type, f.type_name = _F.TYPE_MESSAGE, f".{PACKAGE}.{typ[2:]}"
            elif typ.startswith("E:"):
                f.type, f.type_name = _F.TYPE_ENUM, f".{PACKAGE}.{typ[2:]}"
            else:
                f.type = _TYPES[typ]
            if label == "optional":           # proto3 explicit presence: synthetic oneof
                oneof = f"_{name}"
                f.proto3_optional = True
            if oneof is not None:
                if oneof not in oneofs:
                    oneofs[oneof] = len(msg.oneof_decl)
                    msg.oneof_decl.add(name=oneof)
                f.oneof_index = oneofs[oneof]
    for svc, methods in SERVICES.items():
        s = fd.service.add(name=svc)
        for mname, (req, resp) in methods.items():
            s.method.add(name=mname, input_type=f".{PACKAGE}.{req}", output_type=f".{PACKAGE}.{resp}")
    return fd


_POOL = descriptor_pool.DescriptorPool()
_FILE = _POOL.Add(_build_file())


class _Messages:
    """Attribute access to the generated message classes (``pb.Tensor`` ...)."""

    def __getattr__(self, name: str):
        cls = message_factory.GetMessageClass(_POOL.FindMessageTypeByName(f"{PACKAGE}.{name}"))
        setattr(self, name, cls)
        return cls


pb = _Messages()
MessageType = {n: i for i, n in enumerate(MESSAGE_TYPES)}


def file_descriptor_proto() -> descriptor_pb2.FileDescriptorProto:
    return _build_file()


# ---------------------------------------------------------------------------
# tensors
# ---------------------------------------------------------------------------
_DTYPES = {"float32": np.float32, "float64": np.float64, "int64": np.int64}


def tensor_to_proto(t, dim_names: Optional[Sequence[str]] = None):
    a = t.detach().cpu().numpy() if isinstance(t, torch.Tensor) else np.asarray(t)
    if a.dtype.name not in _DTYPES:
        raise TypeError(f"unsupported wire dtype {a.dtype}")
    msg = pb.Tensor(dtype=a.dtype.name, tensor_content=np.ascontiguousarray(a).tobytes())
    for i, s in enumerate(a.shape):
        d = msg.tensor_shape.dim.add(size=int(s))
        if dim_names is not None:
            d.name = dim_names[i]
    return msg


def proto_to_numpy(msg) -> np.ndarray:
    shape = tuple(d.size for d in msg.tensor_shape.dim)
    return np.frombuffer(msg.tensor_content, dtype=_DTYPES[msg.dtype]).reshape(shape).copy()


def proto_to_tensor(msg) -> torch.Tensor:
    return torch.from_numpy(proto_to_numpy(msg))


# ---------------------------------------------------------------------------
# state_dict <-> ModelUpdate
# ---------------------------------------------------------------------------
def _state_keys() -> List[str]:
    keys = ["prior_mean", "prior_variance", "beta", "topic_word_matrix",
            "inf_net.input_layer.weight", "inf_net.input_layer.bias",
            "inf_net.hiddens.l_0.0.weight", "inf_net.hiddens.l_0.0.bias"]
    for head in ("inf_net.f_mu", "inf_net.f_sigma"):
        keys += [f"{head}.weight", f"{head}.bias"]
        keys += [f"{head}_batchnorm.{s}" for s in ("running_mean", "running_var", "num_batches_tracked")]
    keys += [f"beta_batchnorm.{s}" for s in ("running_mean", "running_var", "num_batches_tracked")]
    keys += ["best_components", "inf_net.adapt_bert.weight", "inf_net.adapt_bert.bias"]
    return keys


# state_dict key <-> ModelUpdate field: '.' -> '_' except the first hidden layer
_KEY_TO_FIELD = {k: k.replace(".", "_") for k in _state_keys()}
_KEY_TO_FIELD["inf_net.hiddens.l_0.0.weight"] = "inf_net_hiddens_l00_weight"
_KEY_TO_FIELD["inf_net.hiddens.l_0.0.bias"] = "inf_net_hiddens_l_00_bias"
_FIELD_TO_KEY = {f: k for k, f in _KEY_TO_FIELD.items()}
assert sorted(_FIELD_TO_KEY) == sorted(_MODEL_UPDATE_FIELDS)


def key_to_field(key: str) -> str:
    if key not in _KEY_TO_FIELD:
        raise ValueError(f"state_dict key {key!r} has no ModelUpdate field (the reference schema "
                         "carries one hidden-to-hidden layer and no label head)")
    return _KEY_TO_FIELD[key]


def field_to_key(field: str) -> str:
    return _FIELD_TO_KEY[field]


def model_update_from_state(state: Dict[str, Any], current_epoch: int = -1):
    mu = pb.ModelUpdate(current_epoch=current_epoch)
    for k, v in state.items():
        getattr(mu, key_to_field(k)).CopyFrom(tensor_to_proto(v))
    return mu


def state_from_model_update(mu) -> Dict[str, torch.Tensor]:
    out = {}
    for f in _MODEL_UPDATE_FIELDS:
        if mu.HasField(f):
            t = proto_to_tensor(getattr(mu, f))
            out[field_to_key(f)] = t
    return out


def updates_from_state(state: Dict[str, Any]) -> list:
    """``repeated Update`` of a ClientTensorRequest (tensor_name = state_dict key)."""
    return [pb.Update(tensor_name=k, tensor=tensor_to_proto(v)) for k, v in state.items()]


def state_from_updates(updates) -> Dict[str, torch.Tensor]:
    return {u.tensor_name: proto_to_tensor(u.tensor) for u in updates}


# ---------------------------------------------------------------------------
# Adam state <-> AdamUpdate
# ---------------------------------------------------------------------------
def adam_update_from_state_dict(sd: Dict) -> Any:
    au = pb.AdamUpdate()
    # the message is Adam's (federated.proto AdamUpdate); other solvers' states have
    # no exp_avg / exp_avg_sq pair and travel as the param group only
    for sid, st in sd.get("state", {}).items():
        if "exp_avg" not in st or "exp_avg_sq" not in st:
            continue
        cs = au.state.contentState.add(state_id=int(sid))
        cs.step.CopyFrom(tensor_to_proto(torch.as_tensor(st["step"], dtype=torch.float32)))
        cs.exp_avg.CopyFrom(tensor_to_proto(st["exp_avg"]))
        cs.exp_avg_sq.CopyFrom(tensor_to_proto(st["exp_avg_sq"]))
    pg = sd["param_groups"][0]
    g = au.paramGroups
    g.lr = float(pg["lr"])
    betas = pg.get("betas", (pg.get("momentum", 0.0), pg.get("alpha", pg.get("rho", 0.0))))
    g.betas.beta1, g.betas.beta2 = float(betas[0]), float(betas[1])
    g.eps, g.weight_decay = float(pg.get("eps", 0.0)), float(pg.get("weight_decay", 0.0))
    g.amsgrad = bool(pg.get("amsgrad", False))
    g.params.extend(int(p) for p in pg["params"])
    return pb.OptUpdate(adamUpdate=au)


def adam_state_dict_from_update(ou) -> Dict:
    au = ou.adamUpdate
    g = au.paramGroups
    state = {}
    for cs in au.state.contentState:
        state[int(cs.state_id)] = {"step": proto_to_tensor(cs.step).reshape(()),
                                   "exp_avg": proto_to_tensor(cs.exp_avg),
                                   "exp_avg_sq": proto_to_tensor(cs.exp_avg_sq)}
    pg = {"lr": g.lr, "betas": (g.betas.beta1, g.betas.beta2), "eps": g.eps,
          "weight_decay": g.weight_decay, "amsgrad": g.amsgrad, "params": list(g.params),
          "maximize": False, "foreach": None, "capturable": False, "differentiable": False,
          "fused": None}
    return {"state": state, "param_groups": [pg]}


# ---------------------------------------------------------------------------
# Dictionary
# ---------------------------------------------------------------------------
def dictionary_from_vocab(vocab: Dict[str, int]):
    d = pb.Dictionary()
    for k, v in vocab.items():
        p = d.pairs.add(key=k)
        p.value.ivalue = int(v)
    return d


def vocab_from_dictionary(d) -> Dict[str, int]:
    return {p.key: int(p.value.ivalue) for p in d.pairs}


def dictionary_from_params(params: Dict[str, Any]):
    """Typed model parameters; floats travel as float32 like the reference."""
    d = pb.Dictionary()
    for k, v in params.items():
        p = d.pairs.add(key=k)
        if v is None:                      # the reference sends None as the string "None"
            p.value.svalue = "None"
        elif isinstance(v, bool):
            p.value.bvalue = v
        elif isinstance(v, (int, np.integer)):
            p.value.ivalue = int(v)
        elif isinstance(v, (float, np.floating)):
            p.value.fvalue = float(v)
        elif isinstance(v, (tuple, list)):
            for x in v:
                p.value.tvalue.values.add(ivalue=int(x))
        else:
            p.value.svalue = str(v)
    return d


def params_from_dictionary(d) -> Dict[str, Any]:
    out = {}
    for p in d.pairs:
        which = p.value.WhichOneof("oneof_values")
        if which == "tvalue":
            out[p.key] = tuple(x.ivalue for x in p.value.tvalue.values)
        elif which == "svalue" and p.value.svalue == "None":
            out[p.key] = None
        elif which is not None:
            out[p.key] = getattr(p.value, which)
    return out
