"""Similarity-graph timing: MFMA tiles vs the numpy float64 restatement.

usage: python tools/bench_similarity.py [--sizes 20000,100000] [--cpu-size 20000] [--out FILE]

Clustered synthetic features (F = 248, like Mutation_feature_248.csv), threshold 0.97.  Reported
per size: the device time of similar_triples (pairs kernel + sort + triples; features already in
HBM), the time of the dominant tile kernel alone, and its f32-MFMA rate on the algorithmic work
(N(N-1)/2 pairs x 2F flop) against the 157.3 TF dense f32 MFMA peak.  The CPU line is the numpy
restatement (oracle/ref_similarity.py, float64 BLAS on the host cores) on --cpu-size nodes.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from iddgcn_amd import ops, similarity  # noqa: E402

PEAK_F32_MFMA = 157.3e12


def features(N, F, seed=0):
    rng = np.random.default_rng(seed)
    centers = rng.standard_normal((max(1, N // 20), F))
    return centers[rng.integers(0, len(centers), N)] + 0.15 * rng.standard_normal((N, F))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="20000,100000")
    ap.add_argument("--cpu-size", type=int, default=20000)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    F, thr = 248, 0.97
    res = {"gpu": [], "cpu": None}
    for N in (int(x) for x in a.sizes.split(",")):
        X = torch.as_tensor(features(N, F), device=dev)
        similarity.similar_triples(X, thr, 3, device=dev)               # warm-up (and capacity sizing)
        keys = ops.similarity_pairs(X, thr)
        cap = int(keys.numel() * 1.1) + 1024
        tt, tp = [], []
        for _ in range(a.reps):
            torch.cuda.synchronize()
            e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            e[0].record()
            k = ops.similarity_pairs(X, thr, capacity=cap)
            e[1].record()
            sk, _ = ops.radix_sort(k, end_bit=int(N * N - 1).bit_length())
            tri = ops.similarity_triples(sk, N, 3, 0)
            e[2].record()
            torch.cuda.synchronize()
            tp.append(e[0].elapsed_time(e[1]))
            tt.append(e[0].elapsed_time(e[2]))
        flop = N * (N - 1) / 2 * 2 * F
        line = {"N": N, "F": F, "threshold": thr, "pairs": int(tri.shape[0]), "total_ms": float(np.median(tt)),
                "pairs_kernel_ms": float(np.median(tp)), "alg_TFLOPs": flop / (np.median(tp) * 1e-3) / 1e12}
        line["mfma_frac"] = line["alg_TFLOPs"] * 1e12 / PEAK_F32_MFMA
        res["gpu"].append(line)
        print(json.dumps(line), flush=True)
        del X, keys, k, sk, tri
        torch.cuda.empty_cache()
    if a.cpu_size:
        from oracle.ref_similarity import similar_triples
        Xc = features(a.cpu_size, F)
        t0 = time.perf_counter()
        ref = similar_triples(Xc, thr, 3, 0)
        dt = time.perf_counter() - t0
        got = similarity.similar_triples(Xc, thr, 3, device=dev)
        res["cpu"] = {"N": a.cpu_size, "seconds": dt, "threads": torch.get_num_threads(),
                      "kind": "port (numpy float64, oracle/ref_similarity.py)", "bit_identical": bool(
                          np.array_equal(ref, got))}
        print(json.dumps(res["cpu"]), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
