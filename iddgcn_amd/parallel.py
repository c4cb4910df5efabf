"""Data parallelism for the full-batch step (one process per GPU, RCCL over xGMI).

Edge partitioning (the default): the scored edges of a full-batch step are
independent given the node tables, so each rank takes a contiguous slice of them; the graph (CSR
of every A_r) and all parameters are replicated.  Every gradient of the step is a sum over scored
edges, so the per-rank gradients — already normalised by the GLOBAL edge count — are summed by an
all-reduce of the flat gradient buffer IN PLACE (FlatParams.buf = [E | rel | layer params | loss]),
after which Adam runs identically on every rank.  There is no other collective on the data path.

The all-reduce is bucketed and overlapped with the end of the backward (BucketedAllReduce): the
small gradients + loss go out as soon as the layer loop ends, then dE in row chunks as the
transposed SpMM finishes each chunk (engine.Engine.backward).
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
            return
        self._works.append(dist.all_reduce(view, op=dist.ReduceOp.SUM, group=self.group, async_op=True))

    def finish(self):
        works, self._works = self._works, []
        for w in works:
            w.wait()

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
