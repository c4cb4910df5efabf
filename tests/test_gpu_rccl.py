"""RCCL itself, executed once on the one-GPU box (VERDICT r04 "RCCL has never executed").

Every multi-rank test runs over gloo (several ranks sharing the one GPU of a builder box), so the collectives the
RCCL ranks of a multi-GPU step issue had never run on RCCL.  A world-size-1 "nccl" process group drives exactly those
calls through RCCL on the box's GPU:

  * ``NodeShard(staged=False)``: padded ``all_gather_into_tensor`` (W^l, X^3 asynchronously) and
    ``reduce_scatter_tensor`` (dO^3 asynchronously, the dWedge head sums);
  * ``BucketedAllReduce``'s device branch: asynchronous in-place ``all_reduce`` of the flat gradient buffer's buckets,
    with ``KerasAdam.apply_overlapped`` updating each bucket as its sum lands (Engine.train_step, edge partitioning);
  * the node-row step's E ownership (round 5, NodeShard owner_e): dE ``reduce_scatter_tensor`` to the row owners,
    ``KerasAdam.apply_owned``, then the asynchronous ``all_gather_into_tensor`` of E (Engine.finish_pending);
  * ``RelationShard``'s ``all_gather_into_tensor`` / ``reduce_scatter_tensor`` (``--shard relation``);
  * the split E collectives (round 6, ``Engine.split_e_collectives``): per-owner ``broadcast`` of E and ``reduce`` of
    dE, the forward's A_r E as one SpMM per source owner (two steps: the second forward takes the broadcast pieces);
  * bench.py's ``rank_consistency`` (broadcast + MAX all-reduce on the device).

With one rank every collective is the identity, so each RCCL step must be BITWISE the same step on a gloo group
(host-staged branches, the one the multi-rank gloo tests check against the full batch), and the edge-partitioned
RCCL step bitwise the step without any communicator.  The child process is fresh (spawned) and joins the nccl group
before it makes any GPU call.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _mild(N, R, D, seed):
    rng = np.random.default_rng(seed)
    p = {"E": rng.standard_normal((N, D)) / np.sqrt(D)}
    for l in (1, 2, 3):
        p[f"K{l}"] = rng.standard_normal((R, D, D)) / D
        p[f"S{l}"] = rng.standard_normal((D, D)) / np.sqrt(D)
        p[f"Wa{l}"] = rng.standard_normal((D, R)) / np.sqrt(D)
        p[f"ba{l}"] = rng.standard_normal(R) * 0.1
    p["rel"] = rng.standard_normal((R, D))
    return {k: v.astype(np.float32) for k, v in p.items()}


def _child(port, q, N, R, D, gemm, features):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    import torch
    import torch.distributed as dist
    # the nccl (RCCL) group first, before any other GPU call of this process
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        sys.path.insert(0, ROOT)
        from bench import rank_consistency
        from iddgcn_amd.engine import Engine, FlatParams, KerasAdam
        from iddgcn_amd.graph import get_adj_mats
        from iddgcn_amd.parallel import BucketedAllReduce, NodeShard, RelationShard, node_ranges, node_shard_triples
        from iddgcn_amd.utils import synthetic_graph
        dev = torch.device("cuda", 0)
        gloo = dist.new_group(backend="gloo")
        assert dist.get_backend() == "nccl" and dist.get_backend(gloo) == "gloo"
        pos, neg = synthetic_graph(N, R, 9000, seed=77)
        tri = np.concatenate([pos, neg])
        lab = np.concatenate([np.ones(len(pos)), np.zeros(len(neg))]).astype(np.float32)
        adj = get_adj_mats(pos, N, R, device=dev)
        cuts = node_ranges(np.bincount(tri[:, 2], minlength=N), 1)
        mine, mlab = node_shard_triples(tri, lab, cuts, 0)

        def step(shard, comm, split=False, steps=1):
            eng = Engine(N, R, D, dev, gemm=gemm, features=features)
            eng.split_e_collectives = split
            eng.overlap_e_gather = steps > 1    # E's collectives in flight into the next forward (split: its pieces)
            if shard == "node_rccl":
                eng.row_shard = NodeShard(cuts, staged=False)              # the RCCL ranks' branch
            elif shard == "node_gloo":
                eng.row_shard = NodeShard(cuts, group=gloo, staged=True)   # host-staged, as the gloo tests
            elif shard == "relation_rccl":
                eng.node_shard = RelationShard(R, N)
            elif shard == "relation_gloo":
                eng.node_shard = RelationShard(R, N, group=gloo)
            ed = eng.edges(mine, mlab) if shard.startswith("node") else eng.edges(tri, lab)
            P, G = FlatParams(N, R, D, dev), FlatParams(N, R, D, dev)
            P.load(_mild(N, R, D, 9))
            opt = KerasAdam(P)
            for _ in range(steps):
                loss = eng.train_step(P, G, opt, adj, ed, t_global=len(tri), comm=comm)
            eng.finish_pending()        # node rows (owner_e): the all-gather of E the step left in flight
            torch.cuda.synchronize()
            return float(loss.item()), G.buf.cpu().numpy(), P.buf.cpu().numpy(), P.buf

        res = {}
        res["plain"] = step("none", None)
        res["edge_rccl"] = step("none", BucketedAllReduce(min_bucket_rows=64))          # nccl: async device buckets
        res["node_rccl"] = step("node_rccl", BucketedAllReduce(min_bucket_rows=64))
        res["node_gloo"] = step("node_gloo", BucketedAllReduce(group=gloo, min_bucket_rows=64))
        res["relation_rccl"] = step("relation_rccl", BucketedAllReduce(min_bucket_rows=64))
        res["relation_gloo"] = step("relation_gloo", BucketedAllReduce(group=gloo, min_bucket_rows=64))
        res["node_rccl_2"] = step("node_rccl", BucketedAllReduce(min_bucket_rows=64), steps=2)
        res["node_rccl_split_2"] = step("node_rccl", BucketedAllReduce(min_bucket_rows=64), split=True, steps=2)
        consist = rank_consistency(res["node_rccl"][3])
        q.put(("ok", {k: v[:3] for k, v in res.items()}, consist))
    except BaseException as e:                      # report, then let the process exit non-zero
        q.put(("error", f"{type(e).__name__}: {e}", None))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("N,R,D,gemm,features", [(700, 2, 256, "bf16x3", "f32"), (800, 8, 256, "split", "bf16")])
def test_rccl_world1_collectives_bitwise(N, R, D, gemm, features, cuda):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_child, args=(_free_port(), q, N, R, D, gemm, features))
    p.start()
    status, res, consist = q.get(timeout=240)
    p.join(timeout=60)
    assert status == "ok", res
    assert p.exitcode == 0
    # one rank: every collective is the identity -> bitwise the gloo (host-staged) step, and the edge-partitioned
    # RCCL step (async in-place buckets + bucket-wise Adam) bitwise the step without a communicator
    for a, b in (("edge_rccl", "plain"), ("node_rccl", "node_gloo"), ("relation_rccl", "relation_gloo"),
                 ("node_rccl_split_2", "node_rccl_2")):
        la, ga, pa = res[a]
        lb, gb, pb = res[b]
        assert la == lb, (a, b, la, lb)
        assert np.array_equal(ga, gb), (a, b, "gradients")
        assert np.array_equal(pa, pb), (a, b, "parameters after Adam")
    assert consist == 0.0
    # and the node-partitioned step computes the full batch (its own kernel order: fp32 summation order only)
    lp, gp, _ = res["plain"]
    ln, gn, _ = res["node_rccl"]
    bl, bg = (1e-4, 1e-2) if features == "bf16" else (1e-6, 1e-5)
    assert abs(ln - lp) <= bl * abs(lp)
    assert np.abs(gn - gp).max() <= bg * np.abs(gp).max()
