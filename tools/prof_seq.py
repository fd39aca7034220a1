"""The dispatch sequence of a rocprofv3 kernel-trace database (rocpd SQLite) around its
middle: name, duration and the gap before each dispatch, so one round's order (and what
sits between the kernels: copies, fills, PyTorch ops) can be read off.
usage: python tools/prof_seq.py <results.db> [N=40] [out.md] [anchor]
(anchor: a kernel-name substring; the window starts at its median occurrence)"""
import sqlite3
import sys


def main(db, n="40", out=None, anchor=None):
    n = int(n)
    c = sqlite3.connect(db)
    rows = c.execute("select name, start, end from kernels order by start").fetchall()
    mid = len(rows) // 2
    if anchor:
        hits = [i for i, r in enumerate(rows) if anchor in r[0]]
        if hits:
            mid = hits[len(hits) // 2]
    lines = ["| # | kernel | us | gap before us |", "|---|---|---|---|"]
    for i in range(mid, min(mid + n, len(rows))):
        name, s, e = rows[i]
        gap = (s - rows[i - 1][2]) / 1e3 if i > 0 else 0.0
        lines.append(f"| {i} | {name.split('(')[0][:70]} | {(e - s) / 1e3:.2f} | {gap:.2f} |")
    text = "\n".join(lines)
    print(text)
    if out:
        with open(out, "w") as f:
            f.write(text + "\n")


if __name__ == "__main__":
    main(*sys.argv[1:])
