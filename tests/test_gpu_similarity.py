"""Similarity-graph construction on MFMA (include/iddgcn_similarity.h).

Bar: bit-exact triples (integer output of a float64 threshold decision).
* the reference's bundled features give exactly its bundled outputs mu_similar0.97.csv and
  drug_similar0.78.csv (tests/golden/similarity.npz) — the mutation graph has a pair 1.9e-8 from
  the threshold that f32 alone decides wrongly, so this also exercises the float64 band;
* random clustered features, with pairs planted 1e-7 either side of the threshold, equal the
  float64 oracle (oracle/ref_similarity.py) across partial tiles and odd feature widths;
* edge cases: one node, zero rows, a threshold no pair passes, every pair passing (capacity retry).
"""
import numpy as np
import pytest

from iddgcn_amd import similarity
from iddgcn_amd._lib import IddgcnError
from oracle.ref_similarity import similar_triples as ref_triples

pytestmark = pytest.mark.gpu


def test_bundled_features_reproduce_reference_outputs(cuda, golden):
    g = golden("similarity.npz")
    mu, drug = similarity.feature_relations(g["mu_feat"], g["drug_feat"], device=cuda)
    assert mu.dtype == np.int64 and np.array_equal(mu, g["mu_triples"])
    assert np.array_equal(drug, g["drug_triples"])


def _planted(N, F, thr, seed):
    """Clustered features plus pairs whose cosine sits 1e-7 above / below thr."""
    rng = np.random.default_rng(seed)
    centers = rng.standard_normal((max(1, N // 20), F))
    X = centers[rng.integers(0, len(centers), N)] + 0.15 * rng.standard_normal((N, F))
    for q in range(0, min(N, 40) - 1 if F > 1 else 0, 2):
        u = X[q] / np.linalg.norm(X[q])
        w = rng.standard_normal(F)
        w -= (w @ u) * u
        w /= np.linalg.norm(w)
        c = thr + (1e-7 if q % 4 == 0 else -1e-7)
        X[q + 1] = (c * u + np.sqrt(1 - c * c) * w) * rng.uniform(0.5, 3.0)
    return X


@pytest.mark.parametrize("N,F,thr", [(1000, 248, 0.97), (1000, 248, 0.78), (129, 65, 0.9), (300, 1, 0.5),
                                     (2500, 248, 0.95), (777, 17, 0.99)])
def test_random_features_match_float64_oracle(cuda, N, F, thr):
    X = _planted(N, F, thr, N + F)
    got = similarity.similar_triples(X, thr, 2, 661, device=cuda)
    want = ref_triples(X, thr, 2, 661)
    assert len(want) > 0
    assert np.array_equal(got, want)


def test_edge_cases(cuda):
    rng = np.random.default_rng(0)
    X = rng.standard_normal((1, 8))
    assert similarity.similar_triples(X, 0.5, 3, device=cuda).shape == (0, 3)
    X = rng.standard_normal((200, 30))
    X[[3, 50, 51]] = 0.0                                 # zero rows: norm 1, similarity 0 with everything
    for thr in (-0.5, 0.0, 0.3, 1.0):
        assert np.array_equal(similarity.similar_triples(X, thr, 3, device=cuda), ref_triples(X, thr, 3, 0)), thr
    X = rng.standard_normal((700, 12))
    allp = similarity.similar_triples(X, -2.0, 1, device=cuda)         # every pair: 244,650 > first capacity
    assert len(allp) == 700 * 699 // 2 and np.array_equal(allp, ref_triples(X, -2.0, 1, 0))
    with pytest.raises(IddgcnError):
        similarity.similar_triples(np.array([[1.0, np.nan]]), 0.5, 3, device=cuda)
