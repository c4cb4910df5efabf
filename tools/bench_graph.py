"""Graph-build timing: host numpy build vs the device build, plus the radix sort.

usage: python tools/bench_graph.py [--configs 3,4] [--reps 5] [--out FILE]

For each config the synthetic graph of SURVEY §8(d) (positives + one negative per positive) is
built both ways; host = get_adj_mats + DeviceAdjacency + ScoredEdges (numpy unique/lexsort/argsort,
then H2D), device = DeviceAdjacency.from_triples + ScoredEdges.from_triples with the triples already
in HBM (one H2D of the triples measured separately).  The radix-sort lines give the per-pass
algorithmic bandwidth: a pass reads and writes every key (+ value) once, 2*n*(key+val) bytes.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from iddgcn_amd import ops  # noqa: E402
from iddgcn_amd.graph import DeviceAdjacency, ScoredEdges, get_adj_mats  # noqa: E402
from iddgcn_amd.utils import synthetic_graph  # noqa: E402

CONFIGS = {3: (100_000, 2, 2_000_000), 4: (1_000_000, 2, 20_000_000)}


def timed(fn, reps):
    ts = []
    out = None
    for _ in range(reps):
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        out = fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    return float(np.median(ts)), out


def sort_line(dev, n, kb, end_bit, with_vals, reps):
    rng = np.random.default_rng(0)
    keys = torch.as_tensor(rng.integers(0, 1 << end_bit, n).astype(np.int64 if kb == 8 else np.int32), device=dev)
    ms, _ = timed(lambda: ops.radix_sort(keys, end_bit=end_bit, argsort=with_vals), reps)
    passes = (end_bit + 7) // 8
    vb = 4 if with_vals else 0
    alg = passes * 2 * n * (kb + vb)
    return {"n": n, "key_bytes": kb, "end_bit": end_bit, "values": with_vals, "passes": passes, "ms": ms,
            "keys_per_s": n / ms * 1e3, "alg_GBs": alg / ms / 1e6}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="3,4")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    res = {"sort": [], "build": []}
    for n, kb, eb, v in ((40_000_000, 4, 20, True), (40_000_000, 8, 42, False), (20_000_000, 8, 42, False)):
        res["sort"].append(sort_line(dev, n, kb, eb, v, a.reps))
        print(json.dumps(res["sort"][-1]), flush=True)
    for c in (int(x) for x in a.configs.split(",")):
        N, R, M = CONFIGS[c]
        pos, neg = synthetic_graph(N, R, M, seed=0)
        tri = np.concatenate([pos, neg])
        lab = np.concatenate([np.ones(len(pos), np.float32), np.zeros(len(neg), np.float32)])
        t0 = time.perf_counter()
        host_adj = DeviceAdjacency(get_adj_mats(pos, N, R), N, dev)
        host_ed = ScoredEdges(tri, lab, N, R, dev)
        torch.cuda.synchronize()
        host_s = time.perf_counter() - t0
        t0 = time.perf_counter()
        pos_d = torch.as_tensor(pos, device=dev)
        tri_d = torch.as_tensor(tri, device=dev)
        lab_d = torch.as_tensor(lab, device=dev)
        torch.cuda.synchronize()
        h2d_ms = (time.perf_counter() - t0) * 1e3
        adj_ms, d_adj = timed(lambda: DeviceAdjacency.from_triples(pos_d, N, R, dev), a.reps)
        ed_ms, d_ed = timed(lambda: ScoredEdges.from_triples(tri_d, lab_d, N, R, dev), a.reps)
        same = (torch.equal(d_adj.fwd_col, host_adj.fwd_col) and torch.equal(d_adj.bwd_col, host_adj.bwd_col)
                and torch.equal(d_adj.bwd_ptr, host_adj.bwd_ptr) and torch.equal(d_ed.hperm, host_ed.hperm)
                and torch.equal(d_ed.inv, host_ed.inv))
        line = {"config": c, "N": N, "R": R, "adjacency_edges": len(pos), "scored_edges": len(tri),
                "host_build_s": host_s, "device_adjacency_ms": adj_ms, "device_scored_edges_ms": ed_ms,
                "device_total_ms": adj_ms + ed_ms, "h2d_triples_ms": h2d_ms,
                "speedup_vs_host": host_s * 1e3 / (adj_ms + ed_ms), "bit_identical": bool(same)}
        res["build"].append(line)
        print(json.dumps(line), flush=True)
        del host_adj, host_ed, d_adj, d_ed, pos_d, tri_d, lab_d
        torch.cuda.empty_cache()
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
