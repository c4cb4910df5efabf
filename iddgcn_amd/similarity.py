"""Similarity-graph construction on the GPU (prediction/feat_similarity.py).

The reference script computes ``cosine_similarity(node_feat)`` as a dense float64 matrix,
thresholds it (``creat_similar_mat``) and lists the upper-triangle pairs row-major
(``simat2triple``) as the drug–drug (relation 2) and mutation–mutation (relation 3) edges.
``similar_triples`` does the three steps in one pass over 128×128 MFMA tiles without forming
the N×N matrix (include/iddgcn_similarity.h) and returns the same (M, 3) int64 triples, in the
same order: bit-identical on the reference's bundled features (tests/test_gpu_similarity.py).
"""
import numpy as np
import torch

from . import ops
from ._lib import IddgcnError

MU_THRESHOLD, DRUG_THRESHOLD = 0.97, 0.78       # feat_similarity.py:58-59
MU_RELATION, DRUG_RELATION = 3, 2               # feat_similarity.py:64,66


def similar_triples(node_feat, threshold, relation, start=0, device="cuda", as_numpy=True):
    """caculat_distance -> creat_similar_mat -> simat2triple (feat_similarity.py:9-44).

    node_feat: (N, F) features (numpy / pandas / tensor; rows with NaN must already be dropped, as
    the reference does for drugs at feat_similarity.py:8).  Returns (M, 3) int64
    (i + start, relation, j + start) for i < j with cosine similarity > threshold, row-major."""
    if hasattr(node_feat, "to_numpy"):
        node_feat = node_feat.to_numpy()
    X = node_feat if isinstance(node_feat, torch.Tensor) else torch.as_tensor(np.asarray(node_feat, np.float64))
    X = X.to(device=device, dtype=torch.float64).contiguous()
    if X.dim() != 2 or X.shape[0] == 0 or X.shape[1] == 0:
        raise IddgcnError(f"node_feat must be a non-empty (N, F) matrix, got {tuple(X.shape)}")
    if bool(torch.isnan(X).any()):
        raise IddgcnError("node_feat has NaN rows (drop them first, feat_similarity.py:8)")
    N = X.shape[0]
    keys = ops.similarity_pairs(X, threshold)
    end_bit = max(1, int(N * N - 1).bit_length())
    skeys, _ = ops.radix_sort(keys, end_bit=end_bit)
    tri = ops.similarity_triples(skeys, N, relation, start)
    return tri.cpu().numpy() if as_numpy else tri


def feature_relations(mu_feat, drug_feat, device="cuda"):
    """The script's driver (feat_similarity.py:58-67): (mutation triples, drug triples)."""
    mu = similar_triples(mu_feat, MU_THRESHOLD, MU_RELATION, 0, device)
    drug = similar_triples(drug_feat, DRUG_THRESHOLD, DRUG_RELATION, len(mu_feat), device)
    return mu, drug
