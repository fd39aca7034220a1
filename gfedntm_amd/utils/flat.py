"""One flat fp32 buffer for every floating-point tensor of a model's state.

Why: the per-round FedAvg of the reference serializes ~20 tensors per client
into protobuf and averages them one by one in numpy on the server
(reference src/federation/server.py:442-521).  On MI355X the whole shared
state is one contiguous HBM buffer, pre-scaled by w_i = n_i / sum(n) and
summed by a single RCCL all-reduce over xGMI, in place.  The nn.Module keeps
working unchanged: its parameters and BN running buffers become *views* into
the flat buffer, so ``state_dict()`` / ``load_state_dict()`` / the wire format
are untouched.

Layout: tensors listed in ``shared`` (the ``grads_to_share`` keys present in
the model) come first, in state_dict order, so the collective covers one
prefix ``flat[:n_shared]``; the remaining float tensors follow.  Every tensor
starts at a multiple of 32 floats (128 B, a cache line): kernels use 16-B vector loads,
and the large-vocabulary update kernels' tile blocks (64 words of W_in, rows of
adapt_bert) then start on a line.

``transposed`` names 2-D weights stored column-major ([in, out] row-major):
``inf_net.input_layer.weight`` is [H0, V] in PyTorch but the sparse encoder
gathers one *column* per non-zero token, so it is stored as [V, H0] and the
module sees the ``.t()`` view.

``padded`` maps 2-D weights to a row-stride multiple: the fused engine's
``{"beta": BETA_PAD}`` (64, ops/engine.py) stores the [K, V] topic-word matrix with rows of
``round_up(V, 64)`` floats (256 B), so every row starts on a cache line and a row is whole
64-column tiles -- the pipelined large-V backward (bwd_pre = 3) requires ``ld % 64 == 0``
and stores a partial last tile's columns into the padding.  The fused large-vocabulary kernels read-modify-write beta, Adam
m and v in 64-column tiles; with rows of V = 112 027 floats each tile row straddles
three cache lines and the same RMW stream ran at 3.4 instead of 5.0 TB/s
(``profiles/r3/adam_rmw_alignment.jsonl``).  The module sees the [K, V] slice of the
padded [K, ld] storage (a strided view); the pad columns are zero and stay zero (zero
gradients, Adam steps of zero, FedAvg of zeros).
"""
from __future__ import annotations

import dataclasses
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import torch
from torch import nn

ALIGN = 32


@dataclasses.dataclass
class Slot:
    key: str
    offset: int
    shape: Tuple[int, ...]
    numel: int                  # storage floats (rows x ld for a padded slot)
    transposed: bool
    is_param: bool
    ld: int = 0                 # storage row stride of a padded 2-D slot (0: unpadded)


def slot_view(buf: torch.Tensor, s: Slot, storage: bool = False) -> torch.Tensor:
    """The tensor of slot ``s`` inside a flat-layout buffer: the module-shaped view, or
    with ``storage`` the contiguous storage-order one ([in, out] for a transposed weight,
    [rows, ld] for a padded one)."""
    flat = buf[s.offset: s.offset + s.numel]
    if s.transposed:
        t = flat.view(s.shape[1], s.shape[0])
        return t if storage else t.t()
    if s.ld:
        t = flat.view(s.shape[0], s.ld)
        return t if storage else t[:, : s.shape[1]]
    return flat.view(s.shape)


def _resolve(module: nn.Module, key: str):
    *path, leaf = key.split(".")
    owner = module
    for p in path:
        owner = getattr(owner, p)
    return owner, leaf


class FlatState:
    def __init__(self, model: nn.Module, shared_keys: Sequence[str] = (),
                 transposed: Iterable[str] = (), device=None, shared_last: Sequence[str] = (),
                 padded: Optional[Dict[str, int]] = None):
        self.model = model
        sd = model.state_dict(keep_vars=True)
        params = dict(model.named_parameters())
        float_keys = [k for k, v in sd.items() if v.is_floating_point()]
        shared = [k for k in float_keys if k in set(shared_keys)]
        # ``shared_last`` keys close the shared prefix (the fused engine overlaps the
        # all-reduce of a tail range that is final early in the step)
        shared = [k for k in shared if k not in shared_last] + [k for k in shared_last if k in shared]
        rest = [k for k in float_keys if k not in set(shared)]
        self.transposed = set(transposed)
        self.slots: Dict[str, Slot] = {}
        off = 0
        padded = padded or {}
        for k in shared + rest:
            t = sd[k]
            off = -(-off // ALIGN) * ALIGN
            ld, numel = 0, t.numel()
            if k in padded and t.dim() == 2 and k not in self.transposed:
                ld = -(-t.shape[1] // padded[k]) * padded[k]
                off = -(-off // padded[k]) * padded[k]      # rows aligned as well
                numel = t.shape[0] * ld
            self.slots[k] = Slot(k, off, tuple(t.shape), numel, k in self.transposed,
                                 k in params, ld)
            off += numel
        last_shared = self.slots[shared[-1]] if shared else None
        self.n_shared = 0 if last_shared is None else last_shared.offset + last_shared.numel
        self.n_total = -(-off // ALIGN) * ALIGN
        device = device if device is not None else next(iter(sd.values())).device
        self.buffer = torch.zeros(self.n_total, dtype=torch.float32, device=device)
        self.shared_keys = shared
        self.int_keys = [k for k, v in sd.items() if not v.is_floating_point()]
        for k in shared + rest:
            src = sd[k].detach()
            view = self.view(k)
            view.copy_(src.to(view.device, torch.float32))
            owner, leaf = _resolve(model, k)
            if k in params:
                p = getattr(owner, leaf)
                p.data = view
            else:
                owner._buffers[leaf] = view

    def view(self, key: str) -> torch.Tensor:
        return slot_view(self.buffer, self.slots[key])

    def view_like(self, buf: torch.Tensor, key: str) -> torch.Tensor:
        """The slot of ``key`` inside another buffer with this layout (gradients)."""
        return slot_view(buf, self.slots[key])

    def shared_buffer_slots(self) -> List[Slot]:
        """Shared float tensors that are not parameters (batch-norm running stats)."""
        return [self.slots[k] for k in self.shared_keys if not self.slots[k].is_param]

    def raw(self, key: str) -> torch.Tensor:
        """Storage-order (contiguous) view: [in, out] for transposed weights, [rows, ld]
        for padded ones."""
        return slot_view(self.buffer, self.slots[key], storage=True)

    @property
    def shared(self) -> torch.Tensor:
        return self.buffer[: self.n_shared]

    def param_slots(self) -> List[Slot]:
        return [s for s in self.slots.values() if s.is_param]

    def param_ranges(self) -> List[Tuple[int, int]]:
        """Contiguous [start, end) ranges covering all parameters (for flat Adam)."""
        out: List[Tuple[int, int]] = []
        for s in sorted(self.param_slots(), key=lambda s: s.offset):
            a, b = s.offset, s.offset + s.numel
            if out and -(-out[-1][1] // ALIGN) * ALIGN == a:
                out[-1] = (out[-1][0], b)
            else:
                out.append((a, b))
        return out

    def param_mask(self) -> torch.Tensor:
        """1.0 where the flat buffer holds a parameter element, else 0.0."""
        m = torch.zeros(self.n_total, dtype=torch.float32, device=self.buffer.device)
        for s in self.param_slots():
            m[s.offset: s.offset + s.numel] = 1.0
        return m

    def state_dict_subset(self, keys: Optional[Sequence[str]] = None) -> Dict[str, torch.Tensor]:
        sd = self.model.state_dict()
        keys = list(sd.keys()) if keys is None else [k for k in keys if k in sd]
        return {k: sd[k] for k in keys}
