"""numpy restatement of prediction/feat_similarity.py (similarity-graph construction).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).  The reference script runs at import time
(reads Windows paths, writes CSVs), so its functions are restated here:

* caculat_distance  feat_similarity.py:9-12   sklearn cosine_similarity: rows divided by their L2
                                              norm (a zero norm counts as 1), then X·Xᵀ, float64
* creat_similar_mat feat_similarity.py:23-27  mat > threshold -> 1
* simat2triple      feat_similarity.py:35-44  (i + start, relation, j + start) for i < j, row-major
* the driver        feat_similarity.py:58-71  mutations: rel 3, start 0, threshold 0.97;
                                              drugs (NaN rows dropped): rel 2, start 661, 0.78

Pinned: reproduces the reference's bundled outputs mu_similar0.97.csv and drug_similar0.78.csv
exactly (tests/test_oracle.py; tests/golden/similarity.npz holds inputs and expected triples).
"""
import numpy as np


def caculat_distance(node_feat):
    x = np.asarray(node_feat, dtype=np.float64)
    n = np.sqrt(np.einsum("ij,ij->i", x, x))
    n[n == 0] = 1.0
    xn = x / n[:, None]
    return xn @ xn.T


def creat_similar_mat(mat, threshold):
    out = np.zeros_like(mat)
    out[mat > threshold] = 1
    return out


def simat2triple(mat, relation, start):
    i, j = np.nonzero(np.triu(np.asarray(mat) != 0, 1))     # row-major, i < j
    return np.stack([i + start, np.full_like(i, relation), j + start], 1).astype(np.int64)


def similar_triples(node_feat, threshold, relation, start):
    return simat2triple(creat_similar_mat(caculat_distance(node_feat), threshold), relation, start)
