"""Per-workgroup wall time of the gathered forward row GEMM (rowgemm256_b3_kernel<2>) in a real config-3 training step:
the instrumented library (tools/runs/dbg/wgt.so: s_memrealtime at each workgroup's start and end, NV = 2 launches
only, so the table holds the step's last one: the layer-3 forward) runs one engine step built as bench.py builds it.
Prints the spread of workgroup durations per column half and the per-range tile costs (distinct tails per tile).

usage: python tools/runs/dbg/wg_times.py tools/runs/dbg/wgt.so
"""
import ctypes
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from bench import CONFIGS, reference_init  # noqa: E402
from iddgcn_amd import _lib as L  # noqa: E402
from iddgcn_amd.engine import Engine, FlatParams, KerasAdam  # noqa: E402
from iddgcn_amd.graph import get_adj_mats  # noqa: E402
from iddgcn_amd.utils import synthetic_graph  # noqa: E402
from tools.bench_mem import load_lenient  # noqa: E402


def main():
    cfg = CONFIGS[3]
    N, R, D, M = cfg["N"], cfg["R"], cfg["D"], cfg["M"]
    dev = torch.device("cuda", 0)
    pos, neg = synthetic_graph(N, R, M, seed=0)
    tri = np.concatenate([pos, neg])
    lab = np.concatenate([np.ones(len(pos), np.float32), np.zeros(len(neg), np.float32)])
    lib = load_lenient(sys.argv[1])
    L._lib = lib
    eng = Engine(N, R, D, dev, gemm="bf16x3", features="f32")
    adj = get_adj_mats(pos, N, R, device=dev)
    ed = eng.edges(tri, lab)
    P, G = FlatParams(N, R, D, dev), FlatParams(N, R, D, dev)
    P.load(reference_init(np, N, R, D, 89))
    opt = KerasAdam(P)
    for _ in range(3):
        eng.train_step(P, G, opt, adj, ed, t_global=len(tri))
    torch.cuda.synchronize()
    buf = np.zeros(1024 * 4, dtype=np.uint64)
    assert lib.iddgcn_dbg_wgt(ctypes.c_void_p(buf.ctypes.data), ctypes.c_longlong(buf.nbytes)) == 0
    w = buf.reshape(1024, 4).astype(np.int64)
    live = w[:, 1] > 0
    t0 = w[live, 0].min()
    dur = (w[live, 1] - w[live, 0]) / 100.0          # microseconds (100 MHz)
    start = (w[live, 0] - t0) / 100.0
    end = (w[live, 1] - t0) / 100.0
    print(f"workgroups {live.sum()}: start spread {start.min():.1f}-{start.max():.1f} us, duration min/median/max "
          f"{dur.min():.1f} / {np.median(dur):.1f} / {dur.max():.1f} us, last end {end.max():.1f} us")
    q = np.percentile(dur, [5, 25, 50, 75, 95])
    print("duration percentiles 5/25/50/75/95: " + " ".join(f"{v:.1f}" for v in q))
    rng = w[live, 3]
    order = np.argsort(rng)
    slow = np.argsort(dur)[-8:]
    print("slowest ranges (range, tiles, us): " + ", ".join(f"({rng[i]}, {w[live][i, 2]}, {dur[i]:.1f})" for i in slow))
    # distinct tails per tile along the table (the gathered rows each tile DMAs)
    t = ed.t
    if t is not None:
        tt = t[: (len(t) // 32) * 32].view(-1, 32)
        u = 1 + (tt[:, 1:] != tt[:, :-1]).sum(1)
        nr = int(rng.max()) + 1
        per = u.float().cpu().numpy()
        chunks = np.array_split(per, nr)
        print("mean distinct tails per tile by range (first 8, min, max): "
              + " ".join(f"{c.mean():.2f}" for c in chunks[:8]) + f" | {min(c.mean() for c in chunks):.2f} "
              f"{max(c.mean() for c in chunks):.2f}")
    by = {}
    for i in range(len(dur)):
        by.setdefault(int(rng[i]), []).append(dur[i])
    r_sorted = sorted(by)
    print("per-range duration (us), ranges 0..: " + " ".join(f"{np.mean(by[r]):.0f}" for r in r_sorted))


if __name__ == "__main__":
    main()
