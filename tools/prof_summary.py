"""Summarise a rocprofv3 kernel-trace database (rocpd SQLite) into a per-kernel
table: calls, mean / median / total microseconds, and the mean gap between
consecutive kernels of the hot loop.  usage: prof_summary.py <results.db> [out.md]"""
import sqlite3
import sys

import numpy as np


def main(db, out=None):
    c = sqlite3.connect(db)
    rows = c.execute("select name, start, end from kernels order by start").fetchall()
    by = {}
    for n, s, e in rows:
        by.setdefault(n, []).append((e - s) / 1e3)
    lines = ["| kernel | calls | mean us | median us | total ms |", "|---|---|---|---|---|"]
    tot = 0.0
    for n, d in sorted(by.items(), key=lambda kv: -sum(kv[1])):
        d = np.array(d)
        tot += d.sum()
        short = n.split("(")[0][:60]
        lines.append(f"| {short} | {len(d)} | {d.mean():.2f} | {np.median(d):.2f} | {d.sum() / 1e3:.2f} |")
    starts = np.array([r[1] for r in rows], dtype=np.float64)
    ends = np.array([r[2] for r in rows], dtype=np.float64)
    gaps = (starts[1:] - ends[:-1]) / 1e3
    gaps = gaps[(gaps > 0) & (gaps < 50)]
    lines.append("")
    lines.append(f"total kernel time {tot / 1e3:.2f} ms over {len(rows)} dispatches; "
                 f"median inter-kernel gap {np.median(gaps) if len(gaps) else 0:.2f} us")
    text = "\n".join(lines)
    print(text)
    if out:
        with open(out, "w") as f:
            f.write(text + "\n")


if __name__ == "__main__":
    main(*sys.argv[1:])
