"""Device graph build (include/iddgcn_graph.h) against the host build and the oracle.

Integer work, so the bar is bit-exact:
* the radix sort equals numpy's stable sort / argsort (duplicates, partial tiles, every pass count);
* ``DeviceAdjacency.from_triples`` equals the host ``DeviceAdjacency(get_adj_mats(...))`` array for
  array, and its per-relation COO equals oracle/ref_utils.get_adj_coo (utils1.py:420-451),
  on the bundled fold-0 graph and on edge cases (duplicates, an empty relation's (0,0)=0
  placeholder, rows with a relation outside [0, R), no triples, N = 1);
* ``ScoredEdges.from_triples`` equals the host ``ScoredEdges`` (stable tail order, head
  permutation, pointers, inverse, labels);
* a training step on the device-built layouts gives bitwise the same loss and gradients.
"""
import numpy as np
import pytest
import torch

from iddgcn_amd import ops
from iddgcn_amd._lib import IddgcnError
from iddgcn_amd.graph import DeviceAdjacency, ScoredEdges, get_adj_mats
from iddgcn_amd.utils import synthetic_graph
from oracle.ref_utils import get_adj_coo

pytestmark = pytest.mark.gpu


def _np(t):
    return None if t is None else t.cpu().numpy()


@pytest.mark.parametrize("n", [0, 1, 63, 4095, 4096, 4097, 100_003, 1_000_000])
@pytest.mark.parametrize("kind", ["u32", "u64"])
def test_radix_sort_matches_numpy_stable(cuda, n, kind):
    rng = np.random.default_rng(n)
    if kind == "u32":
        keys = rng.integers(0, 1 << 20, n).astype(np.int32)
        end_bit = 20
    else:
        keys = rng.integers(0, 1 << 43, n).astype(np.int64)
        end_bit = 43
    if n > 10:
        keys[: n // 3] = keys[n // 2]                  # a long run of one key: stability matters
    k = torch.as_tensor(keys, device=cuda)
    order = np.argsort(keys, kind="stable")
    ko, vo = ops.radix_sort(k, end_bit=end_bit, argsort=True)
    assert np.array_equal(_np(ko), keys[order])
    assert np.array_equal(_np(vo), order.astype(np.int32))
    vals = rng.integers(0, 1 << 31, n).astype(np.int32)
    ko2, vo2 = ops.radix_sort(k, torch.as_tensor(vals, device=cuda), end_bit=end_bit)
    assert np.array_equal(_np(vo2), vals[order])
    ko3, vo3 = ops.radix_sort(k, end_bit=end_bit)
    assert vo3 is None and np.array_equal(_np(ko3), keys[order])


@pytest.mark.parametrize("end_bit", [0, 1, 7, 8, 9, 16, 17, 32])
def test_radix_sort_bit_ranges(cuda, end_bit):
    rng = np.random.default_rng(end_bit)
    keys = rng.integers(0, 1 << 32, 50_000, dtype=np.uint64).astype(np.uint32)
    keys &= np.uint32((1 << end_bit) - 1) if end_bit < 32 else np.uint32(0xFFFFFFFF)
    k = torch.as_tensor(keys.view(np.int32), device=cuda)
    ko, vo = ops.radix_sort(k, end_bit=end_bit, argsort=True)
    order = np.argsort(keys, kind="stable")
    assert np.array_equal(_np(ko).view(np.uint32), keys[order])
    assert np.array_equal(_np(vo), order.astype(np.int32))


def _same_adjacency(dev, host):
    assert dev.total_nnz == host.total_nnz
    assert dev.nnz == host.nnz
    for name in ("fwd_ptr", "fwd_col", "bwd_ptr", "bwd_col", "bwd_src", "base_values", "fwd_src", "fwd_pos"):
        a, b = _np(getattr(dev, name)), _np(getattr(host, name))
        assert a.dtype == b.dtype and np.array_equal(a, b), name
    for name in ("fwd_val", "bwd_val"):
        a, b = getattr(dev, name), getattr(host, name)
        assert (a is None) == (b is None), name
        if a is not None:
            assert np.array_equal(_np(a), _np(b)), name
    assert np.array_equal(dev.rel_offsets, host.rel_offsets)
    for r in range(host.num_relations):
        assert np.array_equal(dev.rows[r], host.rows[r]) and np.array_equal(dev.cols[r], host.cols[r])


def _check_adjacency(data, N, R, cuda):
    dev = get_adj_mats(data, N, R, device=cuda)
    assert isinstance(dev, DeviceAdjacency)
    host = DeviceAdjacency(get_adj_mats(data, N, R), N, cuda)
    _same_adjacency(dev, host)
    for r, (idx, val) in enumerate(get_adj_coo(np.asarray(data, dtype=np.int64).reshape(-1, 3), N, R)):
        assert np.array_equal(dev.rows[r], idx[:, 0]) and np.array_equal(dev.cols[r], idx[:, 1])
        a, b = dev.rel_offsets[r], dev.rel_offsets[r + 1]
        assert np.array_equal(_np(dev.base_values[a:b]), val)
    return dev


def test_adjacency_fold0_matches_host_and_oracle(cuda, golden):
    d = golden("fold0_data.npz")
    dev = _check_adjacency(d["X_train"], 845, 4, cuda)
    assert dev.nnz == [1482, 1324, 2346, 32358]           # fold-0 nnz per relation
    adj = np.concatenate([d["X_train"], d["X_test"]])      # IDDGCN_eval.py:49 adjacency
    _check_adjacency(adj, 845, 4, cuda)


@pytest.mark.parametrize("case", ["dups", "empty_rel", "foreign_rel", "no_triples", "one_node", "big"])
def test_adjacency_edge_cases(cuda, case):
    rng = np.random.default_rng(7)
    N, R = 300, 3
    if case == "dups":
        tr = rng.integers(0, [N, R, N], (20_000, 3))       # ~20% repeated (h, r, t)
    elif case == "empty_rel":
        tr = rng.integers(0, [N, 2, N], (5_000, 3))        # relation 2 has no edge -> (0,0)=0.0
        tr[:10] = [0, 0, 0]                                # and a real (0,0) in relation 0
    elif case == "foreign_rel":
        tr = rng.integers(0, [N, R + 2, N], (5_000, 3))    # rel >= R rows are ignored, like data[:,1]==i
    elif case == "no_triples":
        tr = np.zeros((0, 3), np.int64)
    elif case == "one_node":
        N = 1
        tr = np.zeros((40, 3), np.int64)
        tr[:, 1] = rng.integers(0, 2, 40)
    else:
        N, R = 100_000, 2
        pos, _ = synthetic_graph(N, R, 2_000_000, seed=0)  # config-3 graph
        tr = pos
    _check_adjacency(tr, N, R, cuda)


def test_adjacency_rejects_out_of_range_entity(cuda):
    tr = np.array([[0, 0, 1], [5, 1, 2]])
    with pytest.raises(IddgcnError):
        get_adj_mats(tr, 5, 2, device=cuda)
    with pytest.raises(IddgcnError):
        get_adj_mats(tr, 5, 2)


def _same_edges(dev, host):
    assert dev.T == host.T
    for name in ("h", "r", "t", "tptr", "hperm", "hptr", "inv", "y"):
        a, b = getattr(dev, name), getattr(host, name)
        assert (a is None) == (b is None), name
        if a is not None:
            assert a.dtype == b.dtype and np.array_equal(_np(a), _np(b)), name


@pytest.mark.parametrize("case", ["fold0", "random", "one", "big"])
def test_scored_edges_match_host(cuda, golden, case):
    N, R = 845, 4
    if case == "fold0":
        d = golden("fold0_data.npz")
        tr = np.concatenate([d["X_train"], d["X_train_neg"]])
        lab = np.concatenate([np.ones(len(d["X_train"])), np.zeros(len(d["X_train_neg"]))])
    elif case == "random":
        rng = np.random.default_rng(3)
        tr = rng.integers(0, [N, R, N], (123_457, 3))
        lab = rng.random(len(tr))
    elif case == "one":
        tr, lab = np.array([[3, 1, 2]]), None
    else:
        N, R = 100_000, 2
        pos, neg = synthetic_graph(N, R, 2_000_000, seed=0)
        tr = np.concatenate([pos, neg])
        lab = np.concatenate([np.ones(len(pos)), np.zeros(len(neg))])
    _same_edges(ScoredEdges.from_triples(tr, lab, N, R, cuda), ScoredEdges(tr, lab, N, R, cuda))


def test_scored_edges_reject_bad_indices(cuda):
    with pytest.raises(IddgcnError, match="entity"):
        ScoredEdges.from_triples(np.array([[0, 0, 9]]), None, 5, 2, cuda)
    with pytest.raises(IddgcnError, match="relation"):
        ScoredEdges.from_triples(np.array([[0, 2, 1]]), None, 5, 2, cuda)


def test_training_step_on_device_built_graph_is_bitwise_equal(cuda):
    from iddgcn_amd.engine import Engine, FlatParams
    N, R, D, M = 2000, 2, 64, 20_000
    pos, neg = synthetic_graph(N, R, M, seed=5)
    rng = np.random.default_rng(0)
    params = {"E": rng.standard_normal((N, D)) / 8}
    for l in (1, 2, 3):
        params.update({f"K{l}": rng.standard_normal((R, D, D)) / D, f"S{l}": rng.standard_normal((D, D)) / 8,
                       f"relw{l}": np.zeros(R), f"Wa{l}": rng.standard_normal((D, R)) / 8, f"ba{l}": np.zeros(R)})
    params["rel"] = rng.standard_normal((R, D))
    params = {k: v.astype(np.float32) for k, v in params.items()}
    tri = np.concatenate([pos, neg])
    lab = np.concatenate([np.ones(len(pos)), np.zeros(len(neg))])
    eng = Engine(N, R, D, cuda)
    out = []
    for adj, ed in ((eng.adjacency(get_adj_mats(pos, N, R)), ScoredEdges(tri, lab, N, R, cuda)),
                    (get_adj_mats(pos, N, R, device=cuda), ScoredEdges.from_triples(tri, lab, N, R, cuda))):
        P, G = FlatParams(N, R, D, cuda), FlatParams(N, R, D, cuda)
        P.load(params)
        loss, p = eng.loss_and_grads(P, G, adj, ed)
        out.append((loss.item(), _np(p), G.to_numpy()))
    assert out[0][0] == out[1][0]
    assert np.array_equal(out[0][1], out[1][1])
    for k in out[0][2]:
        assert np.array_equal(out[0][2][k], out[1][2][k]), k
