"""Topic-model artifacts in the reference npz layout.

Reference: src/utils/auxiliary_functions.py:66-99 (``save_model_as_npz``) and
src/models/federated/federated_model.py:151-197 (``get_results_model`` /
``get_topics_in_server``):

* client file ``{save_client}{id}/model_{id}_{YYYYMMDD}.npz`` -- ``betas`` (K x V
  softmax), ``thetas`` (D x K, values < 3e-3 zeroed then L1-normalised; stored as
  ``thetas_data/indices/indptr/shape`` when sparse), ``ntopics``, ``topics`` (K x 10
  words);
* server file ``{save_server}/global_model_{YYYYMMDD}.npz`` -- ``betas``, ``thetas``
  (None), ``ntopics``, ``topics`` (None).

Everything here writes plain arrays (string topics as a unicode array) so the
files load with ``np.load(allow_pickle=False)``; the reference's ``None`` entries
are written as 0-d object arrays only when explicitly requested for byte parity.
"""
from __future__ import annotations

import datetime
import os
from typing import Optional, Sequence

import numpy as np
import scipy.sparse as sp

THETA_THRESHOLD = 3e-3


def date_stamp(now: Optional[datetime.datetime] = None) -> str:
    return (now or datetime.datetime.now()).strftime("%Y%m%d")


def client_model_path(save_client: str, client_id: int, stamp: Optional[str] = None,
                      epoch: Optional[int] = None) -> str:
    """``{save_client}{id}/model_{id}_{YYYYMMDD}[_epoch_{e}].npz`` (main.py:157)."""
    stamp = stamp or date_stamp()
    name = f"model_{client_id}_{stamp}" + (f"_epoch_{epoch}" if epoch is not None else "")
    return os.path.join(f"{save_client}{client_id}", name + ".npz")


def server_model_path(save_server: str, stamp: Optional[str] = None) -> str:
    """``{save_server}/global_model_{YYYYMMDD}.npz`` (main.py:75)."""
    return os.path.join(save_server, f"global_model_{stamp or date_stamp()}.npz")


def postprocess_thetas(thetas: np.ndarray, threshold: float = THETA_THRESHOLD) -> np.ndarray:
    """Zero entries below ``threshold`` and L1-normalise the rows (federated_model.py:170-173)."""
    t = np.asarray(thetas, dtype=np.float64).copy()
    t[t < threshold] = 0
    s = np.abs(t).sum(axis=1, keepdims=True)
    s[s == 0] = 1.0
    return t / s


def save_model_as_npz(path: str, betas: np.ndarray, thetas, n_components: int,
                      topics: Optional[Sequence[Sequence[str]]]) -> str:
    os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
    payload = {"betas": np.asarray(betas), "ntopics": np.asarray(n_components)}
    if topics is not None:
        payload["topics"] = np.asarray([list(t) for t in topics], dtype=str)
    if sp.issparse(thetas):
        th = sp.csr_matrix(thetas)
        payload.update(thetas_data=th.data, thetas_indices=th.indices, thetas_indptr=th.indptr,
                       thetas_shape=np.asarray(th.shape))
    elif thetas is not None:
        payload["thetas"] = np.asarray(thetas)
    np.savez(path, **payload)
    return path


def load_model_npz(path: str) -> dict:
    """Loads an npz written by :func:`save_model_as_npz` (no pickle)."""
    with np.load(path, allow_pickle=False) as z:
        out = {k: z[k] for k in z.files}
    if "thetas_data" in out:
        out["thetas"] = sp.csr_matrix((out.pop("thetas_data"), out.pop("thetas_indices"),
                                       out.pop("thetas_indptr")), shape=tuple(out.pop("thetas_shape")))
    return out
