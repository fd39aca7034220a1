"""Corpus preprocessing CLI (reference aux_scripts/preprocessing/text_preproc.py).

Non-interactive by default (word lists and thresholds as flags); ``--interactive``
asks for them like the reference.  Writes ``<path_preproc>/iter_<n>/`` with
``corpus.parquet`` (+ ``bow_text``), ``vocabulary.txt`` and ``trainconfig.json``
(see :mod:`gfedntm_amd.data.preprocess`).
"""
from __future__ import annotations

import argparse
import os

from ..data.preprocess import preprocess_parquet


def _ask_files(folder: str, what: str):
    files = sorted(os.listdir(folder))
    for i, f in enumerate(files):
        print(f"{i + 1}. {f}")
    sel = input(f"{what} files (comma-separated numbers): ")
    out = []
    for s in sel.split(","):
        s = s.strip()
        if s.isdigit() and 1 <= int(s) <= len(files):
            out.append(os.path.join(folder, files[int(s) - 1]))
    return out


def main(argv=None):
    p = argparse.ArgumentParser(description="Preprocessing for TM")
    p.add_argument("--path_preproc", required=True)
    p.add_argument("--parquetFile", required=True)
    p.add_argument("--idfld", default="corpusid")
    p.add_argument("--lemmasfld", default="lemmas")
    p.add_argument("--trainer", default="ctm")
    p.add_argument("--iter_", type=int, default=0)
    p.add_argument("--wordlists", default="", help="comma-separated word-list JSON files")
    p.add_argument("--pathWordlists", default=None, help="folder to pick word lists from (--interactive)")
    p.add_argument("--min_lemas", type=int, default=15)
    p.add_argument("--no_below", type=int, default=15)
    p.add_argument("--no_above", type=float, default=0.4)
    p.add_argument("--keep_n", type=int, default=100000)
    p.add_argument("--interactive", action="store_true")
    a = p.parse_args(argv)
    wl = [w for w in a.wordlists.split(",") if w]
    if a.interactive:
        if a.pathWordlists:
            wl += _ask_files(a.pathWordlists, "stopwords")
            wl += _ask_files(a.pathWordlists, "equivalences")
        a.min_lemas = int(input(f"min_lemas ({a.min_lemas}): ") or a.min_lemas)
        a.no_below = int(input(f"no_below ({a.no_below}): ") or a.no_below)
        a.no_above = float(input(f"no_above ({a.no_above}): ") or a.no_above)
        a.keep_n = int(input(f"keep_n ({a.keep_n}): ") or a.keep_n)
    out = os.path.join(a.path_preproc, f"iter_{a.iter_}")
    return preprocess_parquet(a.parquetFile, out, a.idfld, a.lemmasfld, wl, a.min_lemas,
                              a.no_below, a.no_above, a.keep_n, a.trainer)


if __name__ == "__main__":
    main()
