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
    xGMI runs per-link bound rings; a handful of large buckets keeps every ring busy)."""

    def __init__(self, group=None, max_chunks=4, min_bucket_rows=4096):
        self.group = group
        self.max_chunks = max_chunks
        self.min_bucket_rows = min_bucket_rows
        self._works = []
        # a gloo group (CPU collectives, e.g. several ranks sharing one GPU in a test) gets GPU buckets
        # staged through host memory, synchronously; RCCL ("nccl") reduces them in place on the device
        self._host_staged = None

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
