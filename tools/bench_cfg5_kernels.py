"""Time config 5's edge kernels in isolation on the REAL step's buffers (N = 1M, R = 8, T = 50M, bf16 edge tables):
the engine is built as bench.py builds it, one training step fills every table, then each kernel is re-launched
alone with the arguments the step passes it (tail reduction with and without dsum, head backward, DistMult + seeds,
the R = 8 forward edge GEMM), for each library variant given (A/B on identical inputs; outputs compared bitwise
with the first variant's).  Also prints the tail / head segment-length distribution of the workload.

usage: python tools/bench_cfg5_kernels.py [lib.so ...]
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from bench import CONFIGS, reference_init  # noqa: E402
from iddgcn_amd import _lib as L  # noqa: E402
from iddgcn_amd import ops  # noqa: E402
from iddgcn_amd.engine import Engine, FlatParams, KerasAdam  # noqa: E402
from iddgcn_amd.graph import get_adj_mats  # noqa: E402
from iddgcn_amd.sampling import negative_samples  # noqa: E402
from iddgcn_amd.utils import synthetic_graph  # noqa: E402
from tools.bench_mem import load_lenient, timeit  # noqa: E402


def main():
    libs = sys.argv[1:] or [None]
    cfg = CONFIGS[5]
    N, R, D, M = cfg["N"], cfg["R"], cfg["D"], cfg["M"]
    dev = torch.device("cuda", 0)
    pos, _ = synthetic_graph(N, R, M, seed=0)
    neg = negative_samples(pos[::cfg["neg_every"]], N, 89, device=dev)
    tri = np.concatenate([pos, neg])
    lab = np.concatenate([np.ones(len(pos), np.float32), np.zeros(len(neg), np.float32)])
    T = len(tri)
    eng = Engine(N, R, D, dev, gemm=cfg["gemm"], features="bf16")
    adj = get_adj_mats(pos, N, R, device=dev)
    ed = eng.edges(tri, lab)
    P, G = FlatParams(N, R, D, dev), FlatParams(N, R, D, dev)
    P.load(reference_init(np, N, R, D, 89))
    eng.train_step(P, G, KerasAdam(P), adj, ed, t_global=T)
    torch.cuda.synchronize()
    ws = eng.workspace(ed.T, True)
    for name, ptr in (("tail", ed.tptr), ("head", ed.hptr)):
        seg = (ptr[1:] - ptr[:-1]).cpu().numpy()
        q = np.percentile(seg, [50, 90, 99, 99.9])
        print(f"{name} segments: N={len(seg)} mean {seg.mean():.1f} p50/90/99/99.9 {q} max {seg.max()} "
              f"empty {int((seg == 0).sum())}", flush=True)
    do = ws.xt[1]                     # a bf16 edge table with step data (do^2 after the backward)
    cases = {
        "tail_seg R8 bf16": (lambda: ops.tail_seg_reduce(ed.tptr, None, ws.Wedge[1], do, ws.P[1], ws.dP, ws.dWedge),
                             lambda: [ws.dP, ws.dWedge]),
        "tail_seg R8 bf16 +dsum": (lambda: ops.tail_seg_reduce(ed.tptr, None, ws.Wedge[0], do, ws.P[0], ws.dP,
                                                               ws.dWedge, dsum=ws.dES),
                                   lambda: [ws.dP, ws.dWedge, ws.dES]),
        "head_bwd_node": (lambda: ops.head_bwd_node(ws.dOn_a, ws.P[1], ws.Ssm[1], ws.W[1], ws.dP, ws.dz,
                                                    hseg_ptr=ed.hptr, hperm=ed.hperm, dWedge=ws.dWedge),
                          lambda: [ws.dP, ws.dz]),
        "head_bwd_node (no dP)": (lambda: ops.head_bwd_node(ws.dOn_a, ws.P[1], ws.Ssm[1], ws.W[1], None, ws.dz,
                                                            hseg_ptr=ed.hptr, hperm=ed.hperm, dWedge=ws.dWedge),
                                  lambda: [ws.dz]),
        "tail + head (2 passes)": (lambda: (ops.tail_seg_reduce(ed.tptr, None, ws.Wedge[1], do, ws.P[1], ws.dP, ws.dWedge),
                                            ops.head_bwd_node(ws.dOn_a, ws.P[1], ws.Ssm[1], ws.W[1], ws.dP, ws.dz,
                                                              hseg_ptr=ed.hptr, hperm=ed.hperm, dWedge=ws.dWedge)),
                                   lambda: [ws.dP, ws.dz]),
        "tail+head fused": (lambda: (ops.tail_seg_reduce_head(ed.tptr, ws.Wedge[1], do, ws.P[1], ws.dP, ws.dWedge,
                                                               ws.dOn_a, ws.W[1], ws.dwh),
                                     ops.head_dz(ws.Ssm[1], ws.W[1], ed.hptr, ed.hperm, ws.dWedge, ws.dwh, ws.dz)),
                            lambda: [ws.dP, ws.dz]),
        "distmult_heads": (lambda: ops.distmult_bce_heads(ed.hptr, ed.hperm, ws.X[2], ws.xt[2], ed.r, P["rel"], ed.y,
                                                          ws.xt[0], ws.dOn_b, ws.drel_slab, ws.loss_slab,
                                                          scale=1.0 / (T * N)),
                           lambda: [ws.xt[0], ws.dOn_b, ws.loss_slab, ws.drel_slab]),
    }
    x1 = torch.empty_like(ws.xt[0])
    cases["layer-1 tail combine"] = (lambda: ops.combine(ws.ES1, ws.Wedge[0], ws.P[0], x1, y_idx=ed.t, v_idx=ed.t),
                                     lambda: [x1])
    cases["gather_rows W[h]"] = (lambda: ops.gather_rows(ws.W[1], ed.h, ws.Wedge[0]), lambda: [ws.Wedge[0]])
    cases["head_dz"] = (lambda: ops.head_dz(ws.Ssm[1], ws.W[1], ed.hptr, ed.hperm, ws.dWedge, ws.dwh, ws.dz),
                        lambda: [ws.dz])
    dS = torch.empty(D, D, device=dev)
    cases["TN bf16 (dS)"] = (lambda: ops.gemm_tn(ws.xt[0], ws.xt[1], dS, ws.tn_slab), lambda: [dS])
    # the sigma' backward edge GEMM (do^2 . S3^T) * x2 (1 - x2) written to a scratch bf16 table (timing + comparison)
    bwd_out = torch.empty_like(ws.xt[0])
    cases["sigma' bwd GEMM"] = (lambda: ops.rowgemm(ws.xt[1], P["S3"], bwd_out, b_trans=True, act=L.ACT_DSIGMOID,
                                                    aux=ws.xt[0], precision=eng.row_gemm), lambda: [bwd_out])
    cases["sigma' bwd GEMM bf16 ops"] = (lambda: ops.rowgemm(ws.xt[1], P["S3"], bwd_out, b_trans=True,
                                                             act=L.ACT_DSIGMOID, aux=ws.xt[0], precision="bf16"),
                                         lambda: [bwd_out])
    only = os.environ.get("IDDGCN_CFG5_CASES")      # comma-separated case names (and "fwd") to time; default all
    if only:
        cases = {k: v for k, v in cases.items() if k in only.split(",")}
    ref = {}
    for lp in libs:
        if lp:
            L._lib = load_lenient(lp)
        tag = lp.split("/")[-1] if lp else "default"
        for name, (fn, outs) in cases.items():
            ms = timeit(fn, reps=3)
            o = [x.clone() for x in outs()]
            if name not in ref:
                ref[name], same = o, "ref"
            else:
                # (a strided sample of each output for the relative difference: the bf16 edge tables are 25 GB)
                same = "bitwise" if all(torch.equal(a, b) for a, b in zip(o, ref[name])) else \
                    "max rel diff " + ", ".join(
                        f"{((a.flatten()[::97].float() - b.flatten()[::97].float()).abs().max() / b.flatten()[::97].float().abs().max()).item():.2e}"
                        for a, b in zip(o, ref[name]))
            print(f"{tag:14s} {name:24s} {ms:8.3f} ms  {same}", flush=True)
            del o
    # the forward R = 8 edge GEMM (layer 3: x^2 -> x^3, overwritten in place: timing only, after every comparison)
    for lp in (libs if not only or "fwd" in only.split(",") else []):
        if lp:
            L._lib = load_lenient(lp)
        tag = lp.split("/")[-1] if lp else "default"
        for prec, lab in ((eng.row_gemm, "fwd R8 edge GEMM"), ("bf16", "fwd R8 edge GEMM bf16 ops")):
            ms = timeit(lambda: ops.rowgemm(ws.xt[1], P["S3"], ws.xt[2], coef=ws.Wedge[2], V=ws.P[2], v_idx=ed.t,
                                            v_rel_stride=N * D, act=L.ACT_SIGMOID, precision=prec), reps=3)
            print(f"{tag:14s} {lab:24s} {ms:8.3f} ms", flush=True)


if __name__ == "__main__":
    main()
