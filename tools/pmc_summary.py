"""Summarise rocprofv3 ``--pmc`` CSV runs (``run_counter_collection.csv``) into one
per-kernel table: mean counter value per dispatch plus derived ratios.

usage: pmc_summary.py <out.md> <dir1> [<dir2> ...]

Derived columns (gfx950 caveats from the MI355X guide):
  wait%      SQ_WAIT_ANY / SQ_WAVE_CYCLES     (waves parked on s_waitcnt / barriers)
  issue%     SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES (issue stalls: dependencies, pipes)
  active%    SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES
  lds_cf%    SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE (extra cycles from bank conflicts)
  l2_hit%    TCC_HIT_sum / (TCC_HIT_sum + TCC_MISS_sum)
  fetch_kb   FETCH_SIZE (reads ~half the bytes of wide coalesced streams on gfx950)
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def load(dirs):
    vals = defaultdict(lambda: defaultdict(list))      # kernel -> counter -> [per dispatch]
    for d in dirs:
        for path in glob.glob(os.path.join(d, "*counter_collection.csv")):
            with open(path) as f:
                for row in csv.DictReader(f):
                    name = row["Kernel_Name"]
                    for pre in ("void ", "(anonymous namespace)::"):
                        if name.startswith(pre):
                            name = name[len(pre):]
                    name = name.split("(")[0]
                    vals[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return vals


def main(out, dirs):
    vals = load(dirs)
    mean = {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in vals.items()}
    keep = [k for k in mean if k.startswith(("gfk_", "prodlda_", "gfk"))]
    keep.sort(key=lambda k: -mean[k].get("SQ_WAVE_CYCLES", 0))
    pct = lambda a, b: f"{100.0 * a / b:.1f}" if b else "-"  # noqa: E731
    lines = ["| kernel | wave cycles | wait% | issue% | active% | VALU insts | MFMA busy cyc | "
             "LDS active | lds_cf% | fetch KB | write KB | l2_hit% |",
             "|---|---|---|---|---|---|---|---|---|---|---|---|"]
    for k in keep:
        m = mean[k]
        g = lambda c: m.get(c, 0.0)  # noqa: E731
        wc = g("SQ_WAVE_CYCLES")
        lines.append(
            f"| {k[:48]} | {wc:.0f} | {pct(g('SQ_WAIT_ANY'), wc)} | {pct(g('SQ_WAIT_INST_ANY'), wc)} | "
            f"{pct(g('SQ_ACTIVE_INST_ANY'), wc)} | {g('SQ_INSTS_VALU'):.0f} | "
            f"{g('SQ_VALU_MFMA_BUSY_CYCLES'):.0f} | {g('SQ_LDS_IDX_ACTIVE'):.0f} | "
            f"{pct(g('SQ_LDS_BANK_CONFLICT'), g('SQ_LDS_IDX_ACTIVE'))} | {g('FETCH_SIZE'):.1f} | "
            f"{g('WRITE_SIZE'):.1f} | {pct(g('TCC_HIT_sum'), g('TCC_HIT_sum') + g('TCC_MISS_sum'))} |")
    extra = sorted({c for k in keep for c in mean[k]} - {
        "SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_INSTS_VALU",
        "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_LDS_IDX_ACTIVE", "SQ_LDS_BANK_CONFLICT", "FETCH_SIZE",
        "WRITE_SIZE", "TCC_HIT_sum", "TCC_MISS_sum"})
    if extra:
        lines += ["", "| kernel | " + " | ".join(extra) + " |", "|---" * (len(extra) + 1) + "|"]
        for k in keep:
            lines.append(f"| {k[:48]} | " + " | ".join(
                f"{mean[k][c]:.0f}" if c in mean[k] else "-" for c in extra) + " |")
    text = "\n".join(lines) + "\n"
    with open(out, "w") as f:
        f.write(text)
    print(text)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
