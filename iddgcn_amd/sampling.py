"""Negative sampling on the GPU, bit-exact to the reference's host recipe.

``generate_negative_samples_np`` keeps the reference's name, arguments and return value
(prediction/utils1.py:646-655): ``np.random.seed(seed)``, a 0/1 condition per triple and a uniform
entity per triple from numpy's legacy MT19937 stream; the head (condition 1) or the tail (condition 0)
is replaced.  The stream, the masked-rejection ``randint`` and the corruption all run in HIP kernels
(csrc/sampling.hip, include/iddgcn_sampling.h); the arrays returned equal numpy's, element for element.
"""
import numpy as np
import torch

from . import ops
from ._lib import IddgcnError


def negative_samples(triples, num_entities, seed, device=None):
    """(M, 3) negatives of (M, 3) (obj, rel, sbj) triples; GPU tensor in, GPU tensor out (or numpy in,
    numpy out with ``device`` the GPU to use)."""
    if isinstance(triples, torch.Tensor) and triples.is_cuda:
        return ops.negative_samples(triples.to(torch.int64).contiguous(), num_entities, seed)
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    if dev.type != "cuda":
        raise IddgcnError("negative sampling runs on the GPU (no CPU fallback)")
    tr = torch.as_tensor(np.ascontiguousarray(np.asarray(triples, dtype=np.int64).reshape(-1, 3)), device=dev)
    return ops.negative_samples(tr, num_entities, seed).cpu().numpy()


def generate_negative_samples_np(heads, relations, tails, num_entities, seed, device=None):
    """utils1.generate_negative_samples_np: returns (neg_heads, relations, neg_tails) as numpy arrays."""
    heads, relations, tails = (np.asarray(a) for a in (heads, relations, tails))
    if not (heads.shape == relations.shape == tails.shape) or heads.ndim != 1:
        raise IddgcnError("heads, relations and tails must be 1-D arrays of one length")
    neg = negative_samples(np.stack([heads, relations, tails], 1), num_entities, seed, device)
    return neg[:, 0].astype(heads.dtype), relations, neg[:, 2].astype(tails.dtype)
