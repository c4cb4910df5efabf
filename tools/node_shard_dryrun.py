"""Per-rank compute of a node-row partitioned step (parallel.NodeShard), measured on ONE GPU.

For a BASELINE config and a world size W, each rank k's engine (its node range [cuts[k], cuts[k+1]) from
parallel.node_ranges, the scored edges whose tail it owns, the full device adjacency) is built and timed on this
GPU in turn, with the collectives replaced by no-ops (DryShard, DryComm: the rank's Adam included, over the owned E
rows and the all-reduced small weights as in the real step): the kernels run on the rank's true shapes, so the
per-rank time is the compute a rank of a W-GPU job does, without communication.  The single-GPU step is timed
first for reference.  Collective volumes of the real step are reported beside it (bytes per rank), so that
DESIGN.md's strong-scaling model = max_k compute_k + un-overlapped collectives can be written from measurements.
(The numbers the kernels produce here are meaningless - other ranks' rows are never filled - only the timing is.)

usage: python tools/node_shard_dryrun.py [config=4] [world=8] [steps=3] [ranks=all|none|k,k,...] [node_weight]
  (ranks "none": the single-GPU step only; a rank list skips it; node_weight: default parallel.node_row_weight)
"""
import json
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from bench import CONFIGS, reference_init  # noqa: E402
from iddgcn_amd.engine import Engine, FlatParams, KerasAdam  # noqa: E402
from iddgcn_amd.graph import get_adj_mats  # noqa: E402
from iddgcn_amd.parallel import node_ranges, node_row_weight, node_shard_triples  # noqa: E402
from iddgcn_amd.utils import synthetic_graph  # noqa: E402


class _Done:
    def wait(self):
        pass


class DryShard:
    """parallel.NodeShard's interface with the collectives removed (timing only)."""

    def __init__(self, cuts, rank):
        self.cuts, self.rank, self.world = [int(c) for c in cuts], rank, len(cuts) - 1
        self.N = self.cuts[-1]
        self.a, self.b = self.cuts[rank], self.cuts[rank + 1]
        self._idx = None
        self.bytes = 0
        self.owner_e = True         # the node-row step's E ownership (round 5): dE reduce-scattered, Adam over owned rows

    def owned_idx(self, device):
        if self._idx is None:
            self._idx = torch.arange(self.a, self.b, dtype=torch.int32, device=device)
        return self._idx

    def owned_ptr(self, device):
        if getattr(self, "_ptr", None) is None:
            self._ptr = torch.arange(0, self.b - self.a + 1, dtype=torch.int32, device=device)
        return self._ptr

    def all_gather(self, table, async_op=False):
        self.bytes += table.numel() * table.element_size() * (self.world - 1) // self.world
        return _Done()

    def reduce_scatter(self, table, async_op=False):
        self.bytes += table.numel() * table.element_size() * (self.world - 1) // self.world
        return _Done()


class DryComm:
    """parallel.BucketedAllReduce's interface without the all-reduce: the buckets' Adam runs as in a rank's step."""

    def __init__(self, sh):
        self.sh, self._views = sh, []

    def row_chunks(self, n_rows):
        return [(0, n_rows)]

    def ready(self, view):
        self.sh.bytes += 2 * view.numel() * view.element_size() * (self.sh.world - 1) // self.sh.world
        self._views.append(view)

    def finish_each(self, fn):
        views, self._views = self._views, []
        for v in views:
            if fn is not None:
                fn(v)

    def finish(self):
        self.finish_each(None)


def time_steps(eng, P, G, adj, ed, T, steps, comm=None):
    opt = KerasAdam(P)
    eng.train_step(P, G, opt, adj, ed, t_global=T, comm=comm)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        eng.train_step(P, G, opt, adj, ed, t_global=T, comm=comm)
    eng.finish_pending()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3


def main():
    a = sys.argv[1:]
    cid = int(a[0]) if a else 4
    world = int(a[1]) if len(a) > 1 else 8
    steps = int(a[2]) if len(a) > 2 else 3
    only = None if len(a) < 4 or a[3] == "all" else ([] if a[3] == "none" else [int(x) for x in a[3].split(",")])
    cfg = CONFIGS[cid]
    N, R, D, M = cfg["N"], cfg["R"], cfg["D"], cfg["M"]
    feat = cfg.get("features", "f32")
    gemm = cfg.get("gemm", "bf16x3") if feat == "bf16" else "bf16x3"
    dev = torch.device("cuda", 0)
    pos, neg = synthetic_graph(N, R, M, seed=0)
    if cfg.get("neg_every", 1) > 1:
        from iddgcn_amd.sampling import negative_samples
        neg = negative_samples(pos[::cfg["neg_every"]], N, 89, device=dev)
    tri = np.concatenate([pos, neg])
    lab = np.concatenate([np.ones(len(pos), np.float32), np.zeros(len(neg), np.float32)])
    T = len(tri)
    adj = get_adj_mats(pos, N, R, device=dev)
    init = reference_init(np, N, R, D, 89)
    P, G = FlatParams(N, R, D, dev), FlatParams(N, R, D, dev)
    P.load(init)
    out = {"config": cfg["name"], "world": world, "gemm": gemm, "features": feat, "steps": steps}
    eng = Engine(N, R, D, dev, gemm=gemm, features=feat)
    ed = eng.edges(tri, lab)
    if only is None or a[3] == "none":
        out["full_ms"] = time_steps(eng, P, G, adj, ed, T, steps)
        print(json.dumps({"full_ms": out["full_ms"]}), flush=True)
    del eng, ed
    torch.cuda.empty_cache()
    nw = float(a[4]) if len(a) > 4 else node_row_weight(R, feat)
    out["node_weight"] = nw
    cuts = node_ranges(np.bincount(tri[:, 2], minlength=N), world, node_weight=nw)
    out["cuts"] = cuts
    ranks = []
    for k in range(world):
        if only is not None and k not in only:
            continue
        t_k, l_k = node_shard_triples(tri, lab, cuts, k)
        eng = Engine(N, R, D, dev, gemm=gemm, features=feat)
        sh = DryShard(cuts, k)
        eng.row_shard = sh
        ed = eng.edges(t_k, l_k)
        P.load(init)
        ms = time_steps(eng, P, G, adj, ed, T, steps, comm=DryComm(sh))
        r = {"rank": k, "rows": cuts[k + 1] - cuts[k], "scored_edges": int(len(t_k)), "ms": ms,
             "collective_bytes_per_step": sh.bytes // (steps + 1),
             "of_which_dE_reduce_scatter_and_E_all_gather": 2 * (world - 1) * N * D * 4 // world}
        ranks.append(r)
        print(json.dumps(r), flush=True)
        del eng, ed
        torch.cuda.empty_cache()
    out["ranks"] = ranks
    if ranks:
        out["max_rank_ms"] = max(r["ms"] for r in ranks)
        if "full_ms" in out:
            out["compute_speedup"] = out["full_ms"] / out["max_rank_ms"]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
