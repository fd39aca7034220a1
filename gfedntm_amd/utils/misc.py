"""Experiment helpers: Mallet corpus files and the typed experiment-config reader.

Reference: src/aux_modules/utils/misc.py:206-288.  A Mallet import file has one
document per line, ``<id> 0 <text>``.
"""
from __future__ import annotations

import configparser
import contextlib
import gc
import threading
from typing import Any, Dict

_INT_KEYS = {"ntopics", "num_iterations", "batch_size", "num_threads", "optimize_interval",
             "num_epochs", "num_samples", "num_data_loader_workers", "contextual_size",
             "max_features"}
_FLOAT_KEYS = {"thetas_thr", "doc_topic_thr", "alpha", "dropout_in", "dropout_out", "lr",
               "momentum", "topic_prior_mean"}


def mallet_corpus_to_df(corpus_file: str):
    import pandas as pd
    ids, texts = [], []
    with open(corpus_file, encoding="utf-8") as f:
        for line in f:
            head, sep, tail = line.rstrip("\n").partition(" 0 ")
            if not sep:
                continue
            ids.append(head.strip())
            texts.append(tail.strip())
    return pd.DataFrame({"id": ids, "text": texts})


def corpus_df_to_mallet(corpus_df, out_file: str, id_column: str = "id",
                        text_column: str = "text") -> None:
    with open(out_file, "w", encoding="utf-8") as f:
        for i, t in zip(corpus_df[id_column].astype(str), corpus_df[text_column].astype(str)):
            f.write(f"{i} 0 {t}\n")


def read_config_experiments(file_path: str) -> Dict[str, Any]:
    """Flat, typed dict of every option of an experiments INI file."""
    cp = configparser.ConfigParser()
    cp.read(file_path)
    out: Dict[str, Any] = {}
    for section in cp.sections():
        for opt in cp.options(section):
            v = cp.get(section, opt)
            if opt in _INT_KEYS:
                out[opt] = int(v)
            elif opt in _FLOAT_KEYS:
                out[opt] = float(v)
            elif opt == "labels":
                out[opt] = ""
            elif opt == "topic_prior_variance":
                out[opt] = None
            elif opt in ("learn_priors", "reduce_on_plateau"):
                out[opt] = v == "True"
            elif opt == "hidden_sizes":
                out[opt] = tuple(int(x) for x in v.strip()[1:-1].split(",") if x.strip())
            else:
                out[opt] = v
    return out


# One lock per process around graph captures and the device work of request handlers
# that may run on several threads (gRPC clients served from one process): a capture must
# not overlap another thread's device-wide synchronisation.
DEVICE_LOCK = threading.RLock()


@contextlib.contextmanager
def graph_capture(g, **kw):
    """``torch.cuda.graph(g)`` with Python's cyclic GC held off for the capture.

    torch 2.10 no longer collects at capture start, so a GC pass triggered by an
    allocation inside the capture can finalize an unreachable CUDAGraph of an earlier
    engine; destroying its executable graph while a stream captures is illegal and
    aborts the process.  Collect first, then disable the collector until the capture
    ends (the garbage is freed by the next pass).

    The capture mode defaults to ``thread_local``: several engines may live in one
    process on different threads (e.g. gRPC clients served from one process), and in
    the ``global`` mode another thread's ordinary HIP call during this thread's capture
    fails with hipErrorIllegalState."""
    import torch
    kw.setdefault("capture_error_mode", "thread_local")
    with DEVICE_LOCK:
        gc.collect()
        was = gc.isenabled()
        gc.disable()
        try:
            with torch.cuda.graph(g, **kw):
                yield
        finally:
            if was:
                gc.enable()
