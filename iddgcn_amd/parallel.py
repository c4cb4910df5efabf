"""Data parallelism for the full-batch step (one process per GPU, RCCL over xGMI).

The default with more than one GPU is node-row partitioning (NodeShard below; bench.py --shard node).  Rank k owns
a contiguous range of node rows, balanced by tail edges plus node work (node_ranges / node_row_weight), and takes the
scored edges whose TAIL it owns, so every tail-side quantity is local.  The node tables of the owned rows are
computed locally.  What crosses ranks is the head side (W^l and X^3 all-gathered, the head seeds reduce-scattered),
the small weight gradients (all-reduced) and E: dE is reduce-scattered to the row owners, each owner runs Keras Adam
over its rows, and E is all-gathered in per-owner pieces that the next forward consumes as they land
(Engine.forward's owner-split SpMM).

Two alternatives are kept as flags:
  * edge partitioning (``--shard edge``; also IDDGCN_Model.fit's multi-rank branch): each rank takes a contiguous
    slice of the scored edges, the graph and parameters are replicated, and the flat gradient buffer
    [E | rel | layer params | loss] is all-reduced IN PLACE in buckets (BucketedAllReduce) overlapped with the end
    of the backward, after which Adam runs identically on every rank;
  * relation-sharded node tables (RelationShard, ``--shard relation``): the (relation, row) rows of A_r E and P_r^l
    split over the ranks, P^l all-gathered, dP^l reduce-scattered.
"""
import numpy as np
import torch.distributed as dist


def world():
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def shard_range(T, rank, world_size):
    """Contiguous [lo, hi) slice of T scored edges for `rank` (balanced to +-1)."""
    base, rem = divmod(int(T), int(world_size))
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def shard_triples(triples, labels, rank, world_size):
    lo, hi = shard_range(len(triples), rank, world_size)
    return np.asarray(triples)[lo:hi], (None if labels is None else np.asarray(labels)[lo:hi])


class BucketedAllReduce:
    """Sum contiguous pieces of the flat gradient buffer across ranks, in place, as they become final.

    ``ready(view)`` launches an asynchronous all-reduce (SUM) of ``view`` — ordered after every kernel
    already queued on the current stream, so it overlaps whatever is queued next; ``finish()`` makes
    the current stream wait for all of them.  ``row_chunks(N)`` is how the engine splits dE (N rows)
    into buckets: each at least ``min_bucket_rows`` rows, at most ``max_chunks`` of them (RCCL over
    xGMI runs per-link bound rings; a handful of large buckets keeps every ring busy).

    ``host_staged``: None (default) stages GPU buckets through host memory, synchronously, on a gloo group
    (several ranks sharing one GPU in tests) and reduces them in place on the device on RCCL ("nccl");
    False forces the device branch on any backend (gloo's all_reduce takes GPU tensors too, so the tests
    run the asynchronous in-place path the RCCL ranks take); True forces host staging."""

    def __init__(self, group=None, max_chunks=4, min_bucket_rows=4096, host_staged=None):
        self.group = group
        self.max_chunks = max_chunks
        self.min_bucket_rows = min_bucket_rows
        self._works = []
        self._host_staged = host_staged

    def row_chunks(self, n_rows):
        k = max(1, min(self.max_chunks, n_rows // max(1, self.min_bucket_rows)))
        bounds = [n_rows * i // k for i in range(k + 1)]
        return [(bounds[i], bounds[i + 1]) for i in range(k) if bounds[i + 1] > bounds[i]]

    def ready(self, view):
        if not view.numel():
            return
        if self._host_staged is None:
            self._host_staged = dist.get_backend(self.group) == "gloo"
        if self._host_staged and view.is_cuda:
            host = view.cpu()
            dist.all_reduce(host, op=dist.ReduceOp.SUM, group=self.group)
            view.copy_(host)
            self._works.append((None, view))
            return
        self._works.append((dist.all_reduce(view, op=dist.ReduceOp.SUM, group=self.group, async_op=True), view))

    def finish(self):
        self.finish_each(None)

    def finish_each(self, fn):
        """Wait for the buckets in the order they were handed over; after each, ``fn(view)`` (if given) with the
        bucket now summed — work queued there on the current stream overlaps the later buckets' all-reduces
        (the engine's Adam over each bucket's parameter range)."""
        works, self._works = self._works, []
        for w, view in works:
            if w is not None:
                w.wait()
            if fn is not None:
                fn(view)

    def __call__(self, buf):
        """Whole-buffer form (one bucket)."""
        self.ready(buf)
        self.finish()


class RelationShard:
    """Relation-sharded node tables (SURVEY §8(e)'s alternative to edge partitioning, BASELINE config 4's
    "relation-sharded" wording), combined with the edge partitioning of the scored edges.

    The per-relation node tables AE_r = A_r E and P_r^l = AE_r K_r^l are the step's node-level work.  Here
    they are split over the p ranks by flat (relation, node) row r*N + n: rank k computes the rows
    [k*c, (k+1)*c), c = ceil(R*N / p) — whole relations when p divides R (pure relation sharding: R = 8 on
    8 GPUs is one relation per GPU), row blocks of relations otherwise — and the ranks exchange:
      forward   all-gather of P^l (3 x R*N*D floats) so every rank's edge-level work sees every P_r;
      backward  reduce-scatter of dP^l (the edge partial sums) to the owners, which form dK_r (a
                partial over their rows, summed with the other small gradients) and dAE_r (their rows);
                dE = sum_r A_r^T dAE_r then rides in the usual all-reduce of the flat gradient buffer.
    That is ~6 R*N*D floats of collectives per step against edge partitioning's ~N*D (one dE all-reduce)
    in exchange for 1/p of the SpMM and node GEMM work; bench.py --shard relation measures the trade.
    gloo groups (several ranks sharing a GPU in tests) stage the tensors through host memory."""

    def __init__(self, R, N, group=None):
        self.group = group
        self.rank, self.world = dist.get_rank(group), dist.get_world_size(group)
        self.R, self.N = R, N
        self.RN = R * N
        self.chunk = -(-self.RN // self.world)
        self.a = min(self.RN, self.rank * self.chunk)
        self.b = min(self.RN, self.a + self.chunk)
        self._gloo = dist.get_backend(group) == "gloo"

    def pieces(self):
        """(r, n0, n1): the owned rows, per relation."""
        out = []
        for r in range(self.R):
            n0, n1 = max(self.a, r * self.N) - r * self.N, min(self.b, (r + 1) * self.N) - r * self.N
            if n1 > n0:
                out.append((r, n0, n1))
        return out

    def _padded(self, table):
        import torch
        need = self.world * self.chunk
        if need == self.RN:
            return table, False
        return torch.zeros(need, table.shape[1], dtype=table.dtype, device=table.device), True

    def all_gather(self, table):
        """table: [R*N, D] with this rank's rows filled -> every row filled, on every rank."""
        import torch
        full, padded = self._padded(table)
        if padded:
            full[self.a:self.b].copy_(table[self.a:self.b])
        mine = full[self.rank * self.chunk:(self.rank + 1) * self.chunk]
        if self._gloo:
            host = full.cpu()
            parts = list(host.split(self.chunk))
            dist.all_gather(parts, host[self.rank * self.chunk:(self.rank + 1) * self.chunk].clone(), group=self.group)
            full.copy_(torch.cat(parts))
        else:
            dist.all_gather_into_tensor(full, mine, group=self.group)
        if padded:
            table.copy_(full[:self.RN])

    def reduce_scatter(self, table):
        """table: [R*N, D] partial sums on every rank -> this rank's rows hold the sums over ranks."""
        import torch
        full, padded = self._padded(table)
        if padded:
            full[:self.RN].copy_(table)
        mine = full[self.rank * self.chunk:(self.rank + 1) * self.chunk]
        if self._gloo:
            host = full.cpu()
            dist.all_reduce(host, op=dist.ReduceOp.SUM, group=self.group)
            mine.copy_(host[self.rank * self.chunk:(self.rank + 1) * self.chunk])
        else:
            out = torch.empty_like(mine)
            dist.reduce_scatter_tensor(out, full, op=dist.ReduceOp.SUM, group=self.group)
            mine.copy_(out)
        if padded:
            table[self.a:self.b].copy_(full[self.a:self.b])


def node_row_weight(R, features="f32"):
    """Node-level work of one node row in edge-equivalents (scored edges' work), for node_ranges.

    In D x D GEMM rows: a scored edge costs the tail chain's 6 (2 forward, 2 sigma' backward, 2 dS TN), a node row
    9R + 8 (3R + 1 projections, 3R dAE and 3R dK rows, the head chain's 2 forward, 2 backward and 2 dS TN rows, dE's
    1; the SpMM rows and the head / tail reductions scale alike).  The bf16-feature mode halves the edge tables' bytes
    and runs the edge GEMMs at 2 bf16 MFMAs per k-step while the node tables stay fp32: a node row weighs twice as
    many edges.  Calibrated on the single-GPU kernel profiles: R = 2 fp32 (config 4) 4.3, the round-4 constant 4 gave
    per-rank steps within 3% (profiles/r04/dryrun_cfg4.jsonl); R = 8 bf16 (config 5) 26.7 against 26 from the
    node-level vs edge-level kernel times (profiles/r04/kernel_stats_cfg5_r04z4.txt: 79 ms per 1M rows, 151 ms per
    50M scored edges)."""
    return (9.0 * R + 8.0) / 6.0 * (2.0 if features == "bf16" else 1.0)


def node_ranges(tail_counts, world_size, node_weight=4.0):
    """Contiguous node-row ranges [b_k, b_k+1) for a node-partitioned step: balanced by the work a row brings,
    its scored edges (tail segment length) plus ``node_weight`` edge-equivalents of node-level work (the row's
    SpMM, projections and head chain: node_row_weight(R, features); 4 ~ R = 2).  Returns world_size + 1
    boundaries."""
    w = np.asarray(tail_counts, dtype=np.float64) + float(node_weight)
    c = np.concatenate([[0.0], np.cumsum(w)])
    cuts = [int(np.searchsorted(c, c[-1] * k / world_size, side="left")) for k in range(world_size + 1)]
    cuts[0], cuts[-1] = 0, len(w)
    for k in range(1, world_size + 1):          # non-decreasing (empty ranges allowed on tiny graphs)
        cuts[k] = max(cuts[k], cuts[k - 1])
    return cuts


class NodeShard:
    """Node-row partitioning of the step (round 4).

    Rank k owns the node rows [a, b) = [cuts[k], cuts[k+1]) (node_ranges: balanced by tail edges + node work) and
    takes the scored edges whose TAIL it owns.  Everything a tail needs is then local: its layer-1 ES1 row, its
    P_r^l rows (A_r E and the projections over the owned rows only), the tail segment sums of the backward (dP,
    dES).  What crosses ranks, per step (collectives on (N, C) node tables, each rank contributing its rows):
      forward   all-gather W^l (N x R, 3 per step): the dynamic weights of the edges' HEADS;
                all-gather X^3 (N x D): DistMult's head rows;
      backward  reduce-scatter dO^3 (N x D): the head seeds of the rank's edges go to the heads' owners;
                reduce-scatter the dWedge head sums (N x R, 3 per step);
                all-reduce of the flat gradient buffer past E (the weight gradients are partial sums over the owned
                rows / edges);
                dE (the transposed SpMM of the owned dAE rows reaches every column): with ``owner_e`` (default)
                reduce-scattered to the row owners, who alone run Adam over their E rows (1/p of the largest
                update), then E all-gathered, asynchronously, beside the next forward's owner-local start (E S^1 and
                the layer-1 alpha of the owned rows); without it, all-reduced with the rest of the buffer.
    That is 2 N D + 6 N R floats of all-gather / reduce-scatter beside edge partitioning's N D all-reduce, against
    RelationShard's 6 R N D.  Padded to equal chunks (the ranges differ in length); gloo groups (several ranks
    sharing a GPU in tests) stage through host memory."""

    def __init__(self, cuts, group=None, staged=None, owner_e=True):
        self.group = group
        # owner_e (round 5): Engine.train_step reduce-scatters dE to the row owners, runs Adam over the owned E rows only
        # and all-gathers E (instead of all-reducing dE and updating every row on every rank)
        self.owner_e = bool(owner_e)
        self.rank, self.world = dist.get_rank(group), dist.get_world_size(group)
        self.cuts = [int(c) for c in cuts]
        if len(self.cuts) != self.world + 1:
            raise ValueError("NodeShard: one range per rank")
        self.N = self.cuts[-1]
        self.a, self.b = self.cuts[self.rank], self.cuts[self.rank + 1]
        self.cmax = max(self.cuts[k + 1] - self.cuts[k] for k in range(self.world))
        # staged: None = through host memory on a gloo group (several ranks sharing one GPU in tests), the device
        # collectives on RCCL; False = the device collectives (all_gather_into_tensor / reduce_scatter_tensor) on
        # any backend, so that gloo tests on CPU tensors run the code path the RCCL ranks take
        self._gloo = (dist.get_backend(group) == "gloo") if staged is None else bool(staged)
        self._idx = None
        self._ptr = None

    def owned_idx(self, device):
        """int32 arange(a, b) on the device (row indices of the owned range, for gathered-row kernel forms)."""
        import torch
        if self._idx is None or self._idx.device != device:
            self._idx = torch.arange(self.a, self.b, dtype=torch.int32, device=device)
        return self._idx

    def owned_ptr(self, device):
        """int32 arange(0, b - a + 1) on the device: one-entry segments over the owned rows (head_dz reading the
        reduce-scattered head sums ep[a + n] through owned_idx)."""
        import torch
        if self._ptr is None or self._ptr.device != device:
            self._ptr = torch.arange(0, self.b - self.a + 1, dtype=torch.int32, device=device)
        return self._ptr

    def _padded(self, table):
        import torch
        return torch.empty(self.world * self.cmax, *table.shape[1:], dtype=table.dtype, device=table.device)

    def all_gather(self, table, async_op=False):
        """table: (N, C) with this rank's rows [a, b) filled -> every row filled, on every rank.  With ``async_op``
        the collective is only launched (ordered after the work queued so far); the returned handle's ``wait()``
        completes it (the copy of the other ranks' rows into ``table``, ordered on the current stream).  Until
        then the kernels queued in between must not read the other ranks' rows of ``table`` nor write any of
        it."""
        import torch
        n = self.b - self.a
        if self._gloo:
            mine = torch.zeros(self.cmax, *table.shape[1:], dtype=table.dtype)
            mine[:n] = table[self.a:self.b].cpu()
            parts = [torch.empty_like(mine) for _ in range(self.world)]
            dist.all_gather(parts, mine, group=self.group)
            for k in range(self.world):
                a, b = self.cuts[k], self.cuts[k + 1]
                if k != self.rank and b > a:
                    table[a:b].copy_(parts[k][:b - a])
            return _Done()
        full = self._padded(table)
        mine = full[self.rank * self.cmax:(self.rank + 1) * self.cmax]
        mine[:n].copy_(table[self.a:self.b])
        work = dist.all_gather_into_tensor(full, mine, group=self.group, async_op=True)

        def finish():
            work.wait()
            for k in range(self.world):
                a, b = self.cuts[k], self.cuts[k + 1]
                if k != self.rank and b > a:
                    table[a:b].copy_(full[k * self.cmax:k * self.cmax + b - a])
        h = _Pending(finish)
        if not async_op:
            h.wait()
        return h

    def reduce_scatter(self, table, async_op=False):
        """table: (N, C) partial sums on every rank -> this rank's rows [a, b) hold the sums over the ranks (rank
        order; the other rows are left as they were).  ``async_op``: as all_gather (until ``wait()``, the kernels
        queued in between must not touch ``table``)."""
        import torch
        n = self.b - self.a
        if self._gloo:
            host = table.to("cpu", copy=True)    # (a CPU table: .cpu() would alias it)
            dist.all_reduce(host, op=dist.ReduceOp.SUM, group=self.group)
            table[self.a:self.b].copy_(host[self.a:self.b])
            return _Done()
        full = self._padded(table)
        for k in range(self.world):
            a, b = self.cuts[k], self.cuts[k + 1]
            if b > a:
                full[k * self.cmax:k * self.cmax + b - a].copy_(table[a:b])
            if b - a < self.cmax:            # the padding rows take part in the sum: zero them
                full[k * self.cmax + b - a:(k + 1) * self.cmax].zero_()
        out = torch.empty(self.cmax, *table.shape[1:], dtype=table.dtype, device=table.device)
        work = dist.reduce_scatter_tensor(out, full, op=dist.ReduceOp.SUM, group=self.group, async_op=True)

        def finish():
            work.wait()
            table[self.a:self.b].copy_(out[:n])
        h = _Pending(finish)
        if not async_op:
            h.wait()
        return h


    def broadcast_rows(self, table):
        """Every owner's rows [cuts[k], cuts[k+1]) of ``table`` to every rank, one broadcast per owner (split E
        collectives, round 6: the all-gather of E cut by source owner, so that the next forward's A_r E can start on
        the pieces already here).  Issued in owner order on every rank; returns {k: handle}.  Until handle k's
        ``wait()``, kernels must not write rows [cuts[k], cuts[k+1]) nor, for k other than this rank, read them."""
        hs = {}
        for k in range(self.world):
            a, b = self.cuts[k], self.cuts[k + 1]
            if b <= a:
                hs[k] = _Done()
                continue
            if self._gloo:
                host = table[a:b].to("cpu", copy=True)
                dist.broadcast(host, src=k, group=self.group)
                if k != self.rank:
                    table[a:b].copy_(host)
                hs[k] = _Done()
            else:
                work = dist.broadcast(table[a:b], src=k, group=self.group, async_op=True)
                hs[k] = _Pending(work.wait)     # (the own rows: readable at once, writable after wait())
        return hs

    def reduce_rows(self, table, k):
        """Rows [cuts[k], cuts[k+1]) of ``table`` summed over the ranks into rank k's table (split E collectives: the
        reduce-scatter of dE cut by destination owner, each piece issued as soon as the transposed SpMM has written
        it).  Asynchronous on the device path; other ranks' rows of the piece are left undefined for the caller."""
        a, b = self.cuts[k], self.cuts[k + 1]
        if b <= a:
            return _Done()
        if self._gloo:
            host = table[a:b].to("cpu", copy=True)
            dist.all_reduce(host, op=dist.ReduceOp.SUM, group=self.group)
            if k == self.rank:
                table[a:b].copy_(host)
            return _Done()
        if dist.get_backend(self.group) == "gloo":       # (gloo's reduce takes host tensors only)
            work = dist.all_reduce(table[a:b], op=dist.ReduceOp.SUM, group=self.group, async_op=True)
        else:
            work = dist.reduce(table[a:b], dst=k, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
        return _Pending(work.wait)


class _Done:
    def wait(self):
        pass


class _All:
    """Handle over several collective handles: wait() completes them all (idempotent)."""

    def __init__(self, hs):
        self._hs = list(hs)

    def wait(self):
        hs, self._hs = self._hs, []
        for h in hs:
            h.wait()


class _Pending:
    """Handle of an asynchronous NodeShard collective: wait() once completes it (idempotent)."""

    def __init__(self, fn):
        self._fn = fn

    def wait(self):
        if self._fn is not None:
            fn, self._fn = self._fn, None
            fn()


def node_shard_triples(triples, labels, cuts, rank):
    """The scored edges whose tail lies in rank's node range [cuts[rank], cuts[rank+1]) (a NodeShard step), in
    their original order."""
    t = np.asarray(triples)[:, 2]
    keep = (t >= cuts[rank]) & (t < cuts[rank + 1])
    return np.asarray(triples)[keep], (None if labels is None else np.asarray(labels)[keep])
