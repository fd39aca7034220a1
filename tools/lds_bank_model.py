"""LDS bank-conflict attribution by model: every LDS access group of a kernel, written as the
byte address each of the 64 lanes touches, is run through the CDNA4 banking rules
(/opt/skills/guides/MI355X_MICROARCH.md "LDS": lane groups per instruction, bank = dword
address mod 32 or 64, each extra distinct address on a busy bank within a group adds one
LDS-array cycle).  The output is, per access group, the LDS-array cycles of one wave
instruction, the conflict cycles among them, and the instructions per tile, so the kernel's
SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE share measured by rocprofv3 can be attributed to
source lines (the hardware counters have no per-instruction breakdown on this pool).

usage: python tools/lds_bank_model.py [--md out.md]
"""
from __future__ import annotations

import argparse
from collections import defaultdict
from typing import Callable, Dict, List, Optional, Sequence, Tuple

# instruction -> (lane groups, dwords per lane, bank modulus)
_B128_GROUPS = [[*range(0, 4), *range(12, 16), *range(20, 28)],
                [*range(4, 12), *range(16, 20), *range(28, 32)],
                [*range(32, 36), *range(44, 48), *range(52, 60)],
                [*range(36, 44), *range(48, 52), *range(60, 64)]]
INSTR = {
    "ds_read_b32": ([list(range(0, 32)), list(range(32, 64))], 1, 32),
    "ds_read_b64": ([list(range(0, 32)), list(range(32, 64))], 2, 64),
    "ds_read_b128": (_B128_GROUPS, 4, 64),
    "ds_write_b32": ([list(range(0, 32)), list(range(32, 64))], 1, 32),
    "ds_write_b64": ([list(range(g, g + 16)) for g in range(0, 64, 16)], 2, 32),
    "ds_write_b128": ([list(range(g, g + 8)) for g in range(0, 64, 8)], 4, 32),
}


def wave_cycles(instr: str, addr: Sequence[Optional[int]]) -> Tuple[int, int]:
    """(LDS-array cycles, conflict cycles) of one wave instruction; addr[lane] = byte
    address of the lane's first dword, None for an inactive lane."""
    groups, nd, mod = INSTR[instr]
    total = extra = 0
    for g in groups:
        banks: Dict[int, set] = defaultdict(set)
        for lane in g:
            a = addr[lane]
            if a is None:
                continue
            for d in range(nd):
                dw = a // 4 + d
                banks[dw % mod].add(dw)
        # a group needs (its dwords / the banks' width) cycles at best; each extra distinct
        # dword on a bank adds one
        worst = max((len(s) for s in banks.values()), default=1)
        total += worst
        extra += worst - 1
    return total, extra


Access = Tuple[str, str, Callable[[int, int], Optional[int]], int]   # name, instr, f(wave, lane), count


def run(name: str, accesses: List[Access], waves: int) -> List[dict]:
    rows = []
    for label, instr, f, count in accesses:
        tot = ext = 0
        for w in range(waves):
            c, e = wave_cycles(instr, [f(w, ln) for ln in range(64)])
            tot += c
            ext += e
        rows.append(dict(kernel=name, access=label, instr=instr, per_tile=count,
                         cycles=tot * count, conflict=ext * count))
    return rows


# ---------------------------------------------------------------------------------------
# csrc/prodlda.hip prodlda_bwd_pipe_kernel (K-range workgroup, 8 waves, per tile)
LDP = 72


def _dtt_swz(c):
    return ((c >> 2) & 7) << 2


def pipe_accesses(nks: int = 4) -> List[Access]:
    NTH, RPQ = 512, 32
    A: List[Access] = []
    thT, bt, dt, dtT = 0, 64 * LDP, 128 * LDP, 192 * LDP
    RQ = (nks + 1) // 2
    # staging: beta slice quads, dlogit quads, dlogit^T scalars
    A.append(("bt store (b128)", "ds_write_b128",
              lambda w, l: 4 * (bt + ((64 * w + l) >> 4) * LDP + 4 * ((64 * w + l) & 15)), RQ))
    A.append(("dt store (b128)", "ds_write_b128",
              lambda w, l: 4 * (dt + ((64 * w + l) >> 4) * LDP + 4 * ((64 * w + l) & 15)), 2))
    for e in range(4):
        A.append((f"dtT store e={e} (b32)", "ds_write_b32",
                  lambda w, l, e=e: 4 * (dtT + (4 * ((64 * w + l) & 15) + e) * LDP
                                         + (((64 * w + l) >> 4) ^ _dtt_swz(4 * ((64 * w + l) & 15) + e))), 2))

    # mm64 operand reads: row base + 16 q + g4 (^ swizzle), 4 b128 per operand per subtile
    def mm_read(base_row, swz):
        def f(w, l, q=0):
            r, g4 = l & 15, 4 * (l >> 4)
            row = base_row(w, r)
            return 4 * (row * LDP + ((16 * q + g4) ^ (swz(row) if swz else 0)))
        return f
    ndt = -(-(4 * nks) // 8)
    A.append(("dtheta A: dt rows (b128)", "ds_read_b128", mm_read(lambda w, r: 128 + (w % 4) * 16 + r, None), 4 * ndt))
    A.append(("dtheta B: bt rows (b128)", "ds_read_b128", mm_read(lambda w, r: 64 + (w // 4) * 16 + r, None), 4 * ndt))
    mu = -(-(nks * 4) // 8)
    A.append(("dbeta A: thT rows (b128)", "ds_read_b128", mm_read(lambda w, r: (w >> 2) * 16 + r, None), 4 * mu))
    A.append(("dbeta B: dtT rows (b128, swizzled)", "ds_read_b128",
              lambda w, l: 4 * (dtT + ((w & 3) * 16 + (l & 15)) * LDP
                                + ((4 * (l >> 4)) ^ _dtt_swz((w & 3) * 16 + (l & 15)))), 4 * mu))
    # G tile: stores (b32, XOR 16 (k & 4)) and row-wise quad reads
    for e in range(4):
        A.append((f"G store e={e} (b32)", "ds_write_b32",
                  lambda w, l, e=e: 4 * (dtT + ((w >> 2) * 16 + (l >> 4) * 4 + e) * 64
                                         + ((((w & 3) * 16 + (l & 15))) ^ (((((w >> 2) * 16 + (l >> 4) * 4 + e)) & 4) << 2))), mu))
    A.append(("G read (b128)", "ds_read_b128",
              lambda w, l: 4 * (dtT + ((64 * w + l) >> 4) * 64 + ((4 * ((64 * w + l) & 15)) ^ (((((64 * w + l) >> 4)) & 4) << 2))), RQ))
    A.append(("Adam: beta quads (b128)", "ds_read_b128",
              lambda w, l: 4 * (bt + ((64 * w + l) >> 4) * LDP + 4 * ((64 * w + l) & 15)), RQ))
    return A


# ---------------------------------------------------------------------------------------
# csrc/posterior.hip: LDS-staged batch matrices [B][K], 16 lanes (a DPP row) per column
def post_accesses(K: int, B: int = 64, ld: Optional[int] = None) -> List[Access]:
    ld = ld or K
    rpt = B // 16
    A: List[Access] = []
    # post_colstats_dpp: lane (c = tid >> 4, g = tid & 15) reads rows g + 16 i of column c
    for i in range(rpt):
        A.append((f"colstats row block {i} (b32)", "ds_read_b32",
                  lambda w, l, i=i: 4 * (((l & 15) + 16 * i) * ld + (4 * w + (l >> 4)) % (2 * K)), 1))
    return A


# ---------------------------------------------------------------------------------------
# csrc/update.hip win_tile_ctx: G = A^T dz over the batch rows (A role: at rows, B role: dz)
def winctx_accesses(H0: int, B: int = 64, stride_a: int = 64, stride_z: Optional[int] = None) -> List[Access]:
    sz = stride_z or H0
    at0 = B * sz
    return [("A role: adapted rows (b32)", "ds_read_b32",
             lambda w, l: 4 * (at0 + (l >> 4) * stride_a + (w % 4) * 16 + (l & 15)), B // 4),
            ("B role: dz0 rows (b32)", "ds_read_b32",
             lambda w, l: 4 * ((l >> 4) * sz + (w // 4) * 16 + (l & 15)), B // 4)]


def table(rows: List[dict]) -> str:
    out = ["| kernel | access group | instruction | per tile | LDS cycles | conflict cycles |",
           "|---|---|---|---|---|---|"]
    for r in rows:
        out.append(f"| {r['kernel']} | {r['access']} | {r['instr']} | {r['per_tile']} | "
                   f"{r['cycles']} | {r['conflict']} |")
    by: Dict[str, List[int]] = defaultdict(lambda: [0, 0])
    for r in rows:
        by[r["kernel"]][0] += r["cycles"]
        by[r["kernel"]][1] += r["conflict"]
    out.append("")
    out.append("| kernel | LDS cycles | conflict cycles | conflict share |")
    out.append("|---|---|---|---|")
    for k, (c, e) in by.items():
        out.append(f"| {k} | {c} | {e} | {100.0 * e / max(c, 1):.1f} % |")
    return "\n".join(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--md", default=None)
    a = ap.parse_args()
    rows = []
    rows += run("prodlda_bwd_pipe K=200 (nks 4)", pipe_accesses(4), 8)
    rows += run("prodlda_bwd_pipe K=100 (nks 2)", pipe_accesses(2), 8)
    rows += run("post colstats K=50 (LDS)", post_accesses(50), 16)
    rows += run("post colstats K=100 (LDS)", post_accesses(100), 16)
    rows += run("post colstats K=100, rows at 114", post_accesses(100, ld=114), 16)
    rows += run("win_tile_ctx H0=50, strides 64 / 50", winctx_accesses(50), 8)
    rows += run("win_tile_ctx H0=50, strides 80 / 80", winctx_accesses(50, stride_a=80, stride_z=80), 8)
    md = table(rows)
    print(md)
    if a.md:
        with open(a.md, "w") as f:
            f.write(md + "\n")


if __name__ == "__main__":
    main()
