"""Edge-partitioned data parallelism (one process per GPU, RCCL over xGMI).

The scored edges of a full-batch step are independent given the node tables,
so each rank takes a contiguous slice of them; the graph (CSR of every A_r)
and all parameters are replicated.  Every gradient of the step is a sum over
scored edges, so the per-rank gradients — already normalised by the GLOBAL
edge count — are summed with ONE all-reduce of the flat gradient buffer
(plus the loss partial riding along in the same call), after which Adam runs
identically on every rank.  There is no other collective on the data path.
"""
import numpy as np
import torch
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


class GradAllReduce:
    """Sum the flat gradient buffer and the loss partial across ranks in one call.

    The loss scalar is appended to a persistent bucket that aliases nothing, so
    the collective moves |grads| + 1 floats.
    """

    def __init__(self, flat_grads, group=None):
        self.group = group
        self.bucket = torch.empty(flat_grads.numel() + 1, dtype=flat_grads.dtype, device=flat_grads.device)

    def __call__(self, flat_grads, loss):
        n = flat_grads.numel()
        self.bucket[:n].copy_(flat_grads)
        self.bucket[n:].copy_(loss.view(-1))
        dist.all_reduce(self.bucket, op=dist.ReduceOp.SUM, group=self.group)
        flat_grads.copy_(self.bucket[:n])
        loss.copy_(self.bucket[n:])
