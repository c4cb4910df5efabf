"""Explainers on the GPU against the explainer oracle (oracle/ref_explain.py, float64 autograd of the
reference formulation), fold 4 with the bundled weights and the reference's test triples.

Bars: p within 4x the fp32 oracle's deviation (floor 1e-6; the trained weights saturate the
sigmoids, fp32 drifts ~1e-5 from fp64); value gradients within 4x the fp32 oracle's deviation from fp64 (floor 1e-5 of
max|g|); explaiNE: our top-k scores equal the oracle's to 2e-4 of the largest (fp32 drifts ~4e-5 here), triples identical where scores are separated; mask explainers:
final masked values within 1e-5, top-k triples identical where scores are separated.
"""
import numpy as np
import pytest
import torch

from iddgcn_amd import get_IDDGCN_Model
from iddgcn_amd import explain as X
from iddgcn_amd.graph import DeviceAdjacency, get_adj_mats
from oracle import ref_explain
from oracle.ref_utils import get_adj_coo

pytestmark = pytest.mark.gpu
N_ENT, N_REL = 845, 4


def _setup(golden):
    d, ex, w = golden("fold4_data.npz"), golden("explain_fold4.npz"), golden("weights_fold4.npz")
    model = get_IDDGCN_Model(N_ENT, N_REL, 64, 64, 123, None, 0, 4)
    model.load_weights("tests/golden/weights_fold4.npz")
    adjacency = np.concatenate([d["X_train"].astype(np.int64), ex["test_triples"]])
    return model, w, adjacency, ex["test_triples"]


def test_value_grads_match_oracle(golden, cuda):
    model, w, adjacency, test = _setup(golden)
    eng, P = model._device_state(), model._params
    dadj = DeviceAdjacency(get_adj_mats(adjacency, N_ENT, N_REL), N_ENT, cuda)
    coo = get_adj_coo(adjacency, N_ENT, N_REL)
    for tr in test[:4]:
        dv, p = eng.value_grads(P, dadj, eng.edges(tr[None]))
        p64, g64 = ref_explain.value_grads(w, tr, coo)
        p32, g32 = ref_explain.value_grads(w, tr, coo, dtype=torch.float32)
        assert abs(float(p[0]) - p64) <= max(4 * abs(p32 - p64), 1e-6)
        ours = np.concatenate([g.cpu().numpy() for g in dv]).astype(np.float64)
        ref, r32 = np.concatenate(g64), np.concatenate(g32).astype(np.float64)
        scale = np.abs(ref).max()
        fp32_dev = np.abs(r32 - ref).max() / scale
        err = np.abs(ours - ref).max() / scale
        assert err <= max(4 * fp32_dev, 1e-5), (tr, err, fp32_dev)


def test_masked_values_and_placeholder(golden, cuda):
    """set_values (adj * sigmoid(mask)) == rebuilding the adjacency with those values; a relation
    absent from the computation graph keeps TF's (0,0)=0 placeholder."""
    model, w, adjacency, test = _setup(golden)
    eng, P = model._device_state(), model._params
    tr = test[0]
    comp = X.get_computation_graph(tr[0], tr[1], tr[2], adjacency)
    mats = get_adj_mats(comp, N_ENT, N_REL)
    rng = np.random.default_rng(0)
    vals = [rng.random(m.nnz).astype(np.float32) * m.values for m in mats]
    a = DeviceAdjacency(mats, N_ENT, cuda)
    a.set_values(torch.as_tensor(np.concatenate(vals), device=cuda))
    for m, v in zip(mats, vals):
        m.values = v
    b = DeviceAdjacency(mats, N_ENT, cuda)
    ed = eng.edges(tr[None])
    pa, pb = eng.predict(P, a, ed), eng.predict(P, b, ed)
    assert torch.equal(pa, pb)
    coo = [(np.stack([m.rows, m.cols], 1), v) for m, v in zip(mats, vals)]
    p64, _ = ref_explain.value_grads(w, tr, coo)
    p32, _ = ref_explain.value_grads(w, tr, coo, dtype=torch.float32)
    assert abs(float(pa[0]) - p64) <= max(4 * abs(p32 - p64), 1e-6)


def _check_topk(our_p, our_s, ref_p, ref_s, tol):
    np.testing.assert_allclose(np.sort(our_s)[::-1], np.sort(ref_s)[::-1], rtol=0, atol=tol)
    sep = np.ones(len(ref_s), bool)
    gaps = np.abs(np.diff(ref_s)) > tol
    sep[:-1] &= gaps
    sep[1:] &= gaps
    assert np.array_equal(our_p[sep], ref_p[sep])


def test_explaine_matches_oracle(golden, cuda):
    model, w, adjacency, test = _setup(golden)
    ours_p, ours_s = X.explaine(model, adjacency, test[:6], top_k=10)
    ref_p, ref_s = ref_explain.explaine(w, adjacency, test[:6], N_ENT, N_REL, top_k=10)
    for k in range(6):
        _check_topk(ours_p[k], ours_s[k], ref_p[k], ref_s[k], 2e-4 * np.abs(ref_s[k]).max())


def test_explaine_graph_replay_equals_eager(golden, cuda):
    """The HIP-graph path (device-side single-edge layout + torch.sort ranking, replayed per triple)
    returns bitwise the eager path's scores and the same triples, over 12 consecutive triples."""
    model, w, adjacency, test = _setup(golden)
    ge_p, ge_s = X.explaine(model, adjacency, test[:12], top_k=10, graph=False)
    gr_p, gr_s = X.explaine(model, adjacency, test[:12], top_k=10, graph=True)
    assert np.array_equal(gr_s, ge_s)
    assert np.array_equal(gr_p, ge_p)


@pytest.mark.parametrize("kind", ["gnnexplainer", "iddgcn"])
def test_mask_explainers_match_oracle(kind, golden, cuda):
    """GnnExplainer.py (5 epochs, thr .2) and IDDGCN_explain.py (10 epochs, thr .15, ratio loss), three
    triples in a row: the shared Adam's state carries over between triples as in the reference."""
    model, w, adjacency, test = _setup(golden)
    init = np.random.default_rng(123).standard_normal((N_ENT, N_ENT)).astype(np.float32)
    kw = dict(num_epochs=5, threshold=0.2) if kind == "gnnexplainer" else dict(
        num_epochs=10, threshold=0.15, target_ratios=(0.4, 0.4, 0.1, 0.1))
    ours_p, ours_s, ours_m = X.mask_explainer(model, adjacency, test[:3], init_value=init, return_masks=True, **kw)
    ref_p, ref_s, ref_m = ref_explain.mask_explainer(w, adjacency, test[:3], N_ENT, N_REL, init, **kw)
    for k in range(3):
        np.testing.assert_allclose(ours_m[k], ref_m[k], rtol=0, atol=1e-5)
        _check_topk(ours_p[k], ours_s[k], ref_p[k], ref_s[k], 1e-5)
