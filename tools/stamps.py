"""Diagnostic: per-phase cycle counts inside the fused-step kernels (s_memtime stamps).

Builds a -DGFK_STAMPS copy of the kernel library into build/stamps/, runs a few
eager steps of a ProdLDA model of the given shape on random BoW rows and prints the
s_memtime deltas between phase stamps (lane 0 of workgroup 0; in the vocab-tile loops
of the decoder kernels: the workgroup's last tile).  Read the SHARES, not the
absolute length (the stamps add fences).

(python tools/stamps.py --build-only on the CPU host, then --so build/stamps/... copied
to a travelling path on the GPU box, so the box does not compile)

usage: python tools/stamps.py [--topics K] [--vocab V] [--hidden 50,50] [--batch B]
                              [--nnz N] [--docs D] [--steps S]
"""
import argparse
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def build():
    from tools.build_native import KERNEL_SRCS, KFLAGS
    out = os.path.join(ROOT, "build", "stamps")
    os.makedirs(out, exist_ok=True)
    objs = []
    for s in KERNEL_SRCS:
        src = os.path.join(ROOT, "csrc", s)
        if not os.path.exists(src):
            continue
        o = os.path.join(out, s + ".o")
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950"] + KFLAGS +
                       ["-DGFK_STAMPS", "-c", src, "-o", o], check=True)
        objs.append(o)
    so = os.path.join(out, "libgfedntm_kernels.so")
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-o", so] + objs,
                   check=True)
    return so


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--topics", type=int, default=50)
    p.add_argument("--vocab", type=int, default=4466)
    p.add_argument("--hidden", default="50,50")
    p.add_argument("--batch", type=int, default=64)
    p.add_argument("--nnz", type=int, default=170)
    p.add_argument("--docs", type=int, default=1000)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--ctx", type=int, default=0, help="contextual size: CombinedTM when > 0")
    p.add_argument("--bf16", action="store_true", help="matmul_dtype='bf16' (contextual GEMMs)")
    p.add_argument("--so", default=None, help="a prebuilt -DGFK_STAMPS library (--build-only)")
    p.add_argument("--build-only", action="store_true", help="build it on the host and stop")
    a = p.parse_args(argv)
    if a.build_only:
        print(build())
        return
    so = a.so or build()
    from gfedntm_amd.ops import native
    native.KERNELS_SO = native.KERNELS_SO_OVERRIDE = so    # (a diagnostic build: not hash-checked)
    import torch
    from gfedntm_amd.data.bow import BatchPlan, DeviceCSR
    import numpy as np
    from gfedntm_amd.models import AVITM, CombinedTM
    from tests.helpers import random_csr
    kw = dict(input_size=a.vocab, n_components=a.topics,
              hidden_sizes=tuple(int(h) for h in a.hidden.split(",")), batch_size=a.batch,
              verbose=False, backend="fused", device="cuda")
    if a.bf16:
        kw["matmul_dtype"] = "bf16"
    tm = CombinedTM(contextual_size=a.ctx, **kw) if a.ctx else AVITM(**kw)
    X = random_csr(a.docs, a.vocab, a.nnz, seed=0)
    ctx = (np.random.default_rng(1).standard_normal((a.docs, a.ctx)).astype(np.float32)
           if a.ctx else None)
    data = DeviceCSR(X, "cuda", contextual=ctx)
    tm.engine.bind_data(data, BatchPlan.build(a.docs, a.batch, a.steps))
    dbg = torch.zeros(1024, dtype=torch.int64, device="cuda")
    tm.engine._m.dbg = dbg.data_ptr()
    tm.engine._a.dbg = dbg.data_ptr()
    for s in range(a.steps):
        tm.engine.step(s)
    torch.cuda.synchronize()
    d = dbg.cpu().numpy()
    m = tm.engine._m
    print(f"K={a.topics} V={a.vocab} tiles={m.n_tiles} dec_grid={m.dec_grid} n_dpart={m.n_dpart} "
          f"stage_flags={m.stage_flags}")
    nf = ["stage", "mfma", "bn", "store+rowlse"]
    print("prodlda_fwd (last tile of wg 0) cycles:", {"tile_start->stage": int(d[17] - d[21]),
          **{nf[i]: int(d[17 + i] - d[16 + i]) for i in range(1, 4)}})
    nbw = ["stage", "sparse", "dense+bn_bwd", "mfma+update"]
    print("prodlda_bwd (last tile of wg 0) cycles:", {"stage": int(d[25] - d[23]),
          **{nbw[i]: int(d[25 + i] - d[24 + i]) for i in range(1, 4)}})
    print("post_fwd cycles: stage", int(d[1] - d[0]), "| colstats", int(d[2] - d[1]), "| row", int(d[3] - d[2]))
    print("row_bwd cycles:", int(d[9] - d[8]))
    print("post_bwd cycles: stage", int(d[11] - d[10]), "| colsums", int(d[12] - d[11]), "| rest", int(d[13] - d[12]))
    print("post_bwd rest: wg0 extras", int(d[14] - d[12]), "| bn_bwd", int(d[15] - d[14]),
          "| heads", int(d[29] - d[15]), "| hidden", int(d[13] - d[29]))
    print("enc_in cycles: row+weights issue", int(d[5] - d[4]), "| gather+draws", int(d[6] - d[5]),
          "| input+hidden", int(d[7] - d[6]), "| heads", int(d[39] - d[7]))
    print("enc_in input+hidden: tile-start tail", int(d[44] - d[6]), "| input layer", int(d[43] - d[44]),
          "| hidden layers", int(d[7] - d[43]), "(last layer's gemv+epilogue ends at", int(d[45] - d[43]), ")")
    if a.ctx:
        # (register-streamed forward, the default at large V: prologue = first x phase +
        # ring fill, C loop = the phases' MFMAs, A + P = the epilogue, of wave 0 of wg 0)
        print("ctx_fwd (wg 0) cycles: prologue", int(d[31] - d[30]), "| C loop", int(d[32] - d[31]),
              "| A + P", int(d[33] - d[32]))
        print("ctx_fwd (wg 0) last phase", int(d[32] - d[143]), "| epilogue: first barrier",
              int(d[140] - d[32]), "| A stores + barrier", int(d[141] - d[140]),
              "| split sum", int(d[142] - d[141]), "| P", int(d[33] - d[142]))
        print("ctx_bwd (wg 0) cycles: staging", int(d[35] - d[34]), "| dA", int(d[36] - d[35]),
              "| g_ba + g_Wa", int(d[37] - d[36]), "| update", int(d[38] - d[37]))
    print("win_update (W_in tile 0) cycles: staging", int(d[41] - d[40]), "| mfma+update", int(d[42] - d[41]))
    if m.stage_flags & (1 << 19) and m.lb_fused:
        # the large-batch MFMA decoder (csrc/prodlda.hip prodlda_lb_fwd / _bwd), the last tile
        # of workgroup 0
        print("lb_fwd cycles: beta rows wait", int(d[131] - d[130]), "| mfma", int(d[132] - d[131]),
              "| column stats", int(d[133] - d[132]))
        print("lb_bwd cycles: logit gradient (loads + sparse)", int(d[121] - d[120]),
              "| barrier", int(d[122] - d[121]), "| bn bwd", int(d[123] - d[122]),
              "| dbeta (+ adam)", int(d[124] - d[123]), "| dtheta", int(d[125] - d[124]),
              "| end barrier", int(d[126] - d[125]))
    # strip forward (stage_flags bit 2): per-wave timelines of workgroups 0 and grid - 1,
    # memtime cycles from the earliest wave's entry; clock = memtime / memrealtime (100 MHz)
    for wg, base in (("0", 64), ("last", 320)):
        w = d[base:base + 256].reshape(16, 16)
        if not w[:, 0].any():
            continue
        t0 = w[:, 0].min()
        rt = (w[:, 8] - w[:, 1]).max()
        ghz = (w[:, 7] - w[:, 0]).max() / rt / 10.0 if rt else 0.0
        print(f"strip_fwd wg {wg}: clock {ghz:.2f} GHz (memtime/realtime)")
        for i in range(16):
            r = w[i]
            ev = [("entry", r[0]), ("staged", r[2]), ("mfma0", r[3]), ("mean0", r[9]),
                  ("rstd0", r[10]), ("bnst0", r[11]), ("epi0", r[4]), ("mfma1", r[5]),
                  ("epi1", r[6]), ("end", r[7])]
            print(f"  wave {i:2d}: " + " ".join(f"{n} {int(v - t0)}" for n, v in ev if v))


if __name__ == "__main__":
    main()
