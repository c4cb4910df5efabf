"""Edge-partitioned data parallelism on CPU: world_size 2, gloo backend (no GPU needed).

The product's DP logic is exercised for real: `shard_triples` partitions the scored edges and
`BucketedAllReduce` sums the flat gradient buffer + loss slot IN PLACE, bucket by bucket, in the
order Engine.backward hands the buckets over (all small gradients + loss, then row chunks of dE).
The per-rank compute is the CPU oracle here (the HIP engine needs a GPU; tests/test_gpu_parallel.py
runs the engine itself); each rank normalises by the GLOBAL edge count exactly as
Engine.train_step(t_global=T) does.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from iddgcn_amd.engine import param_layout
from iddgcn_amd.parallel import BucketedAllReduce, shard_range, shard_triples


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle.ref_model import train_step_grads
        from oracle.ref_utils import get_adj_coo
        g = dict(np.load(os.path.join(os.path.dirname(__file__), "golden", "synth_small.npz")))
        N, R = int(g["N"]), int(g["R"])
        params = {k[6:]: v for k, v in g.items() if k.startswith("param_")}
        tri = np.concatenate([g["triples"], g["neg"]])
        lab = np.concatenate([np.ones(len(g["triples"])), np.zeros(len(g["neg"]))])
        my_tri, my_lab = shard_triples(tri, lab, rank, world)
        pos, neg = my_tri[my_lab == 1], my_tri[my_lab == 0]
        adj = get_adj_coo(g["triples"], N, R)            # the graph is replicated on every rank
        loss, _, grads = train_step_grads(params, pos, neg, adj, N)
        D = int(g["D"])
        keys = [name for name, _, _ in param_layout(N, R, D)]           # FlatParams order: E first
        T, Ts = len(tri), len(my_tri)
        buf = torch.cat([torch.as_tensor(grads[k]).reshape(-1) for k in keys] +
                        [torch.tensor([loss * T], dtype=torch.float64)]) * (Ts / T)    # [flat | loss slot]
        comm = BucketedAllReduce(min_bucket_rows=64)
        comm.ready(buf[N * D:])                         # small gradients + loss
        chunks = comm.row_chunks(N)
        assert len(chunks) > 1
        for n0, n1 in chunks:                           # dE row chunks
            comm.ready(buf[n0 * D:n1 * D])
        comm.finish()
        q.put((rank, buf[:-1].numpy(), float(buf[-1]) / T, keys))
    finally:
        dist.destroy_process_group()


def test_shard_range_partitions_exactly():
    for T in (0, 1, 7, 1000, 40316):
        for w in (1, 2, 3, 8):
            parts = [shard_range(T, r, w) for r in range(w)]
            assert parts[0][0] == 0 and parts[-1][1] == T
            assert all(parts[i][1] == parts[i + 1][0] for i in range(w - 1))
            sizes = [b - a for a, b in parts]
            assert max(sizes) - min(sizes) <= 1


def test_dp_world2_gloo_equals_full_batch(golden):
    from oracle.ref_model import train_step_grads
    from oracle.ref_utils import get_adj_coo
    g = golden("synth_small.npz")
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    (_, f0, l0, keys), (_, f1, l1, _) = res
    assert np.array_equal(f0, f1) and l0 == l1                  # identical on every rank after the all-reduce
    full = np.concatenate([g[f"grad_{k}"].reshape(-1) for k in keys])
    assert f0.shape == full.shape
    np.testing.assert_allclose(f0, full, rtol=0, atol=1e-12 * np.abs(full).max() + 1e-18)
    assert abs(l0 - float(g["loss"])) < 1e-12


def test_bucketed_row_chunks_cover_rows():
    c = BucketedAllReduce(max_chunks=4, min_bucket_rows=100)
    for n in (0, 1, 99, 100, 250, 1000, 100_000):
        ch = c.row_chunks(n)
        if n == 0:
            assert ch == []
            continue
        assert ch[0][0] == 0 and ch[-1][1] == n
        assert all(a[1] == b[0] for a, b in zip(ch, ch[1:]))
        assert len(ch) <= 4 and (len(ch) == 1 or min(b - a for a, b in ch) >= 100)


def _shard_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from iddgcn_amd.parallel import RelationShard
        R, N, D = 3, 5, 4
        sh = RelationShard(R, N)
        t = torch.full((R * N, D), -1.0)
        for r, n0, n1 in sh.pieces():
            for n in range(n0, n1):
                t[r * N + n] = r * N + n
        sh.all_gather(t)
        u = torch.ones(R * N, D) * (rank + 1)
        sh.reduce_scatter(u)
        q.put((rank, sh.pieces(), t.numpy(), u.numpy(), sh.a, sh.b))
    finally:
        dist.destroy_process_group()


def test_relation_shard_collectives_world2_gloo():
    """RelationShard (parallel.py): owned (relation, row) pieces partition R*N rows; all_gather fills
    every row on every rank; reduce_scatter leaves the cross-rank sum in the owned rows (R*N = 15 is not
    divisible by 2: the padded path)."""
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_shard_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(2)], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    rows = sorted(r * 5 + n for _, pieces, *_ in res for r, n0, n1 in pieces for n in range(n0, n1))
    assert rows == list(range(15))
    for rank, _, t, u, a, b in res:
        assert np.array_equal(t[:, 0], np.arange(15))
        assert np.all(u[a:b] == 3.0)


def test_node_ranges_balance_and_partition():
    from iddgcn_amd.parallel import node_ranges, node_shard_triples
    rng = np.random.default_rng(3)
    counts = np.concatenate([rng.integers(0, 30, 700), rng.integers(50, 150, 200)])     # mutation / drug tails
    for w in (1, 2, 3, 8):
        cuts = node_ranges(counts, w, node_weight=4.0)
        assert cuts[0] == 0 and cuts[-1] == len(counts) and all(a <= b for a, b in zip(cuts, cuts[1:]))
        work = [counts[a:b].sum() + 4.0 * (b - a) for a, b in zip(cuts, cuts[1:])]
        assert max(work) <= sum(work) / w + 150 + 4.0             # within one row of the balanced share
    tri = np.stack([rng.integers(0, 900, 5000), rng.integers(0, 2, 5000), rng.integers(0, 900, 5000)], 1)
    cuts = node_ranges(np.bincount(tri[:, 2], minlength=900), 3)
    parts = [node_shard_triples(tri, None, cuts, r)[0] for r in range(3)]
    assert sum(len(p) for p in parts) == len(tri)
    for r, p in enumerate(parts):
        assert np.all((p[:, 2] >= cuts[r]) & (p[:, 2] < cuts[r + 1]))


def _node_shard_worker(rank, world, port, q, staged):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from iddgcn_amd.parallel import NodeShard
        cuts = [0, 5, 5, 12][:world + 1] if world == 3 else [0, 7, 12]
        sh = NodeShard(cuts, staged=staged)
        N, C = cuts[-1], 3
        # all-gather: each rank fills its rows with rank-specific values (asynchronously: the handle completes it)
        tab = torch.full((N, C), -1.0)
        tab[sh.a:sh.b] = torch.arange(sh.a, sh.b, dtype=torch.float32)[:, None] * 10 + torch.arange(C)
        h = sh.all_gather(tab, async_op=True)
        h.wait()
        h.wait()                                    # idempotent
        # reduce-scatter: every rank holds partials (rank + 1) * row index; owners get the sums
        part = (rank + 1) * torch.arange(N, dtype=torch.float32)[:, None].repeat(1, C)
        sh.reduce_scatter(part)
        # split E collectives: one broadcast per owner, then one reduce per destination owner (owner rows checked only)
        tb = torch.full((N, C), -1.0)
        tb[sh.a:sh.b] = torch.arange(sh.a, sh.b, dtype=torch.float32)[:, None] * 10 + torch.arange(C)
        hs = sh.broadcast_rows(tb)
        assert sorted(hs) == list(range(world))
        for k in range(world):
            hs[k].wait()
            hs[k].wait()                            # idempotent
        pr = (rank + 1) * torch.arange(N, dtype=torch.float32)[:, None].repeat(1, C)
        for k in range(world):
            sh.reduce_rows(pr, k).wait()
        q.put((rank, tab.numpy(), part[sh.a:sh.b].numpy(), (sh.a, sh.b), part.numpy(), tb.numpy(),
               pr[sh.a:sh.b].numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("staged", [None, False])
@pytest.mark.parametrize("world", [2, 3])
def test_node_shard_collectives_gloo(world, staged):
    """NodeShard.all_gather / reduce_scatter on (N, C) tables with UNEQUAL row ranges (one empty at world 3):
    after the all-gather every rank holds every rank's rows; after the reduce-scatter each owner holds the sums
    of the ranks' partials for its rows and the other rows are untouched.  staged=None: the host-staged gloo
    branch; staged=False: the device branch the RCCL ranks take (padded all_gather_into_tensor with the rank's
    chunk aliased in the output, reduce_scatter_tensor with zeroed padding rows), run here on CPU tensors.  The same
    for the split E collectives (broadcast_rows: every owner's rows to every rank; reduce_rows: each owner's rows
    summed into it)."""
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_node_shard_worker, args=(r, world, port, q, staged)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    N = 12
    want = np.arange(N, dtype=np.float32)[:, None] * 10 + np.arange(3)
    tot = sum(range(1, world + 1))
    for rank, tab, mine, (a, b), part, tb, pr in res:
        assert np.array_equal(tab, want)
        assert np.array_equal(tb, want)
        assert np.array_equal(pr, tot * np.arange(a, b, dtype=np.float32)[:, None].repeat(3, 1))
        assert np.array_equal(mine, tot * np.arange(a, b, dtype=np.float32)[:, None].repeat(3, 1))
        other = np.ones(N, bool)
        other[a:b] = False
        assert np.array_equal(part[other], (rank + 1) * np.arange(N, dtype=np.float32)[other, None].repeat(3, 1))


def _finish_each_worker(rank, world, port, q, host_staged):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        buf = torch.arange(40, dtype=torch.float32) * (rank + 1)
        comm = BucketedAllReduce(host_staged=host_staged)
        pieces = [(30, 40), (0, 10), (10, 20), (20, 30)]      # hand-over order: small part first, then row chunks
        for a, b in pieces:
            comm.ready(buf[a:b])
        seen = []

        def fn(view):
            off = (view.data_ptr() - buf.data_ptr()) // 4
            seen.append((off, off + view.numel(), view.clone().numpy()))

        comm.finish_each(fn)
        q.put((rank, seen, buf.numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("host_staged", [None, False])
def test_bucketed_finish_each_in_order_after_each_sum(host_staged):
    """BucketedAllReduce.finish_each (the hook the overlapped Adam update rides on): the callback sees every bucket
    once, in hand-over order, each already summed over the ranks (gloo world 2 on CPU tensors; host_staged=False:
    the asynchronous in-place branch the RCCL ranks take)."""
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_finish_each_worker, args=(r, 2, port, q, host_staged)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = np.arange(40, dtype=np.float32) * 3
    for _, seen, buf in res:
        assert [(a, b) for a, b, _ in seen] == [(30, 40), (0, 10), (10, 20), (20, 30)]
        for a, b, v in seen:
            assert np.array_equal(v, want[a:b])
        assert np.array_equal(buf, want)
