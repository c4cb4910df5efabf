"""A/B of an Engine switch on a bench config's real buffers: the engine built as bench.py builds it (one training step
first), then whole training steps with ``Engine.<flag>`` True and False alternated (`rounds` rounds of `reps` timed steps
each), medians reported.  Flags: fuse_sigma_tn, fuse_tail_head, overlap (round 6 also timed a merged-dK schedule this way: profiles/r06/ab_merge_dk_cfg5_r06e.txt).

usage: python tools/ab_engine_flag.py --config 5 --flag fuse_sigma_tn [--reps 3] [--rounds 3]
"""
import argparse
import statistics
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from bench import CONFIGS, reference_init  # noqa: E402
from iddgcn_amd.engine import Engine, FlatParams, KerasAdam  # noqa: E402
from iddgcn_amd.graph import get_adj_mats  # noqa: E402
from iddgcn_amd.sampling import negative_samples  # noqa: E402
from iddgcn_amd.utils import synthetic_graph  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=5)
    ap.add_argument("--flag", default="fuse_sigma_tn")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    cfg = CONFIGS[a.config]
    N, R, D, M = cfg["N"], cfg["R"], cfg["D"], cfg["M"]
    dev = torch.device("cuda", 0)
    pos, neg0 = synthetic_graph(N, R, M, seed=0)
    neg = negative_samples(pos[::cfg["neg_every"]], N, 89, device=dev) if "neg_every" in cfg else neg0
    tri = np.concatenate([pos, neg])
    lab = np.concatenate([np.ones(len(pos), np.float32), np.zeros(len(neg), np.float32)])
    T = len(tri)
    eng = Engine(N, R, D, dev, gemm=cfg.get("gemm", "bf16x3"), features=cfg.get("features", "f32"),
                 edge_mfma=cfg.get("edge_mfma", "hilo"))
    adj = get_adj_mats(pos, N, R, device=dev)
    ed = eng.edges(tri, lab)
    del pos, neg, tri, lab
    P, G = FlatParams(N, R, D, dev), FlatParams(N, R, D, dev)
    P.load(reference_init(np, N, R, D, 89))
    opt = KerasAdam(P)
    times = {True: [], False: []}
    for rnd in range(a.rounds):
        for val in (True, False):
            setattr(eng, a.flag, val)
            eng.train_step(P, G, opt, adj, ed, t_global=T)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.reps):
                eng.train_step(P, G, opt, adj, ed, t_global=T)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) / a.reps * 1e3
            times[val].append(ms)
            print(f"round {rnd} config {a.config} {a.flag}={val}: {ms:.2f} ms/step", flush=True)
    for val in (True, False):
        print(f"{a.flag}={val}: median {statistics.median(times[val]):.2f} ms/step over {a.rounds} rounds", flush=True)


if __name__ == "__main__":
    main()
