"""A/B of the fused sigma' backward + dS TN pass (ops.sigma_tn) against the two kernels it replaces, on a bench
config's real buffers (the engine built as bench.py builds it, one training step first): per-launch times (HIP
events, the x table restored before each launch, not timed), the two results compared, then whole training steps
with Engine.fuse_sigma_tn on and off, alternated.
  config 5 (N = 1M, R = 8, T = 50M, bf16 edge tables; ABI 11): gemm_tn256_bf16t_kernel + the v3 sigma' kernel;
  config 3 (N = 100k, R = 2, T = 4M, fp32 tables, bf16x3; ABI 12): gemm_tn256_b3_kernel + rowgemm256_b3_kernel<0, 1>.

usage: python tools/ab_sigma_tn.py [reps] [--config 3|5] [lib.so ...]   (libraries: the fused kernel and the step
timed per build, dx of each compared with the first build's)
"""
import sys
import time

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
from tools.bench_mem import load_lenient  # noqa: E402


def main(reps=5, config=5, libs=()):
    cfg = CONFIGS[config]
    N, R, D, M = cfg["N"], cfg["R"], cfg["D"], cfg["M"]
    dev = torch.device("cuda", 0)
    pos, neg0 = synthetic_graph(N, R, M, seed=0)
    neg = negative_samples(pos[::cfg["neg_every"]], N, 89, device=dev) if "neg_every" in cfg else neg0
    tri = np.concatenate([pos, neg])
    lab = np.concatenate([np.ones(len(pos), np.float32), np.zeros(len(neg), np.float32)])
    T = len(tri)
    feat = cfg.get("features", "f32")
    gemm = cfg.get("gemm", "bf16x3")
    prec = "bf16x3" if feat == "f32" else "exact"
    eng = Engine(N, R, D, dev, gemm=gemm, features=feat)
    adj = get_adj_mats(pos, N, R, device=dev)
    ed = eng.edges(tri, lab)
    P, G = FlatParams(N, R, D, dev), FlatParams(N, R, D, dev)
    P.load(reference_init(np, N, R, D, 89))
    opt = KerasAdam(P)
    eng.train_step(P, G, opt, adj, ed, t_global=T)
    torch.cuda.synchronize()
    ws = eng.workspace(ed.T, True)
    do, x0 = ws.xt[1], ws.xt[0]
    xs = x0.clone()
    S = P["S2"]
    dS_a, dS_b = torch.empty(D, D, device=dev), torch.empty(D, D, device=dev)

    def two():
        ops.gemm_tn(xs, do, dS_a, ws.tn_slab, precision=prec)
        ops.rowgemm(do, S, xs, b_trans=True, act=L.ACT_DSIGMOID, aux=xs, precision=prec)

    def fused():
        ops.sigma_tn(do, xs, S, dS_b, ws.tn_slab, precision=prec)

    libs = list(libs) or [None]

    def timed(fn, label):
        ts = []
        for _ in range(reps):
            xs.copy_(x0)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            fn()
            b.record()
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b))
        print(f"{label:28s} median {np.median(ts):7.3f} ms  runs {' '.join(f'{t:.3f}' for t in ts)}", flush=True)
        return xs[:2_000_000].clone()           # the first 2M rows of dx (a full copy would not fit beside)

    if reps < 0:                                # fused launches only (for a --pmc pass)
        for _ in range(-reps):
            xs.copy_(x0)
            fused()
        torch.cuda.synchronize()
        return
    ref = None
    for rnd in range(2):
        ref = timed(two, f"round {rnd} two kernels")
        for lib in libs:
            if lib:
                L._lib = load_lenient(lib)
            got = timed(fused, f"round {rnd} fused {lib or ''}")
            print(f"   dS max|diff| / max|dS| = {((dS_a - dS_b).abs().max() / dS_a.abs().max()).item():.3e}; "
                  f"dx (first 2M rows) max|diff| / max|dx| = {((ref.double() - got.double()).abs().max() / ref.double().abs().max()).item():.3e}, "
                  f"elements differing {(ref != got).float().mean().item():.3e}", flush=True)
    del xs, ref, got
    for rnd in range(2):
        for lib in [None] + libs:
            if lib:
                L._lib = load_lenient(lib)
            eng.fuse_sigma_tn = lib is not None or libs == [None]
            if lib is None and libs != [None]:
                eng.fuse_sigma_tn = False
            eng.train_step(P, G, opt, adj, ed, t_global=T)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(3):
                eng.train_step(P, G, opt, adj, ed, t_global=T)
            torch.cuda.synchronize()
            print(f"round {rnd} step fuse_sigma_tn={eng.fuse_sigma_tn} {lib or ''}: "
                  f"{(time.perf_counter() - t0) / 3 * 1e3:.1f} ms", flush=True)


if __name__ == "__main__":
    args = sys.argv[1:]
    reps = int(args.pop(0)) if args and args[0].lstrip("-").isdigit() else 5
    config = 5
    if args[:1] == ["--config"]:
        config, args = int(args[1]), args[2:]
    main(reps, config, args)
