"""Data helpers the training / eval scripts call around the hot path.

``generate_reverse_triplets`` (utils1.py:616-623) builds the symmetrised
graph, ``get_y_true`` (utils1.py:657-663) the eval labels, and
``synthetic_graph`` the seeded mutation–drug graphs of SURVEY §8(d).
"""
import numpy as np
import pandas as pd


def generate_reverse_triplets(triplets):
    """utils1.py:616-623: (t, r, h) for every (h, r, t) with h != t."""
    tr = np.asarray(triplets)
    keep = tr[:, 0] != tr[:, 2]
    return tr[keep][:, [2, 1, 0]]


def get_y_true(X_test_pos, X_test_rule):
    """utils1.py:657-663: 1 where a scored triple is a (deduplicated) test positive."""
    pos = pd.DataFrame(np.asarray(X_test_pos)).drop_duplicates()
    rule = pd.DataFrame(np.asarray(X_test_rule))
    merged = pd.merge(rule, pos, indicator=True, how="left")
    return (merged["_merge"] == "both").astype(int).values


def synthetic_graph(num_nodes, num_relations, num_edges, seed=0, mut_frac=661 / 845):
    """Seeded synthetic mutation–drug graph.

    num_edges/2 unique undirected pairs (no self loops) plus their reverses.
    Relations 0/1 are mutation<->drug response edges; relations >= 2 alternate
    drug–drug and mutation–mutation similarity edges.  Returns (M, 3) int64
    triples (obj, rel, sbj) and one negative per edge, corrupting head or tail
    50/50 with a uniform entity (recipe utils1.py:646-655).
    """
    rng = np.random.default_rng(seed)
    n_mut = max(1, int(round(num_nodes * mut_frac)))
    n_drug = max(1, num_nodes - n_mut)
    half = num_edges // 2
    rel = rng.integers(0, num_relations, half * 2)  # oversample, then fill
    heads = np.empty(half * 2, np.int64)
    tails = np.empty(half * 2, np.int64)
    resp = rel < 2
    k = int(resp.sum())
    heads[resp] = rng.integers(0, n_mut, k)
    tails[resp] = n_mut + rng.integers(0, n_drug, k)
    sim = ~resp
    drugdrug = sim & ((rel % 2) == 0)
    mutmut = sim & ((rel % 2) == 1)
    kd, km = int(drugdrug.sum()), int(mutmut.sum())
    heads[drugdrug] = n_mut + rng.integers(0, n_drug, kd)
    tails[drugdrug] = n_mut + rng.integers(0, n_drug, kd)
    heads[mutmut] = rng.integers(0, n_mut, km)
    tails[mutmut] = rng.integers(0, n_mut, km)
    ok = heads != tails
    a, b = np.minimum(heads, tails)[ok], np.maximum(heads, tails)[ok]
    key = (rel[ok] * num_nodes + a) * num_nodes + b
    _, first = np.unique(key, return_index=True)
    first = np.sort(first)[:half]
    if first.size < half:
        raise ValueError("could not draw enough unique pairs; lower num_edges")
    h, r, t = heads[ok][first], rel[ok][first], tails[ok][first]
    pos = np.concatenate([np.stack([h, r, t], 1), np.stack([t, r, h], 1)])
    cond = rng.integers(0, 2, len(pos))
    rnd = rng.integers(0, num_nodes, len(pos))
    neg = pos.copy()
    neg[:, 0] = np.where(cond == 0, pos[:, 0], rnd)
    neg[:, 2] = np.where(cond == 1, pos[:, 2], rnd)
    return pos.astype(np.int64), neg.astype(np.int64)
