"""BASELINE config 4 at FULL size on one GPU (1M nodes, 2 relations, 20M adjacency edges, D=256, 40M scored
edges: T x D edge tables of 41 GB each): the full-batch training step of IDDGCN.py:123-178 with the
relation loop of :68-77, at the size only this configuration reaches — 40M-row edge tables, million-node
tail / head segments, node tables of 1 GB per relation — checked against the float64 oracle
(oracle/ref_model.py) on a 10k scored-edge sample.  The oracle's A_r·E is computed for the sampled edges'
entities only (A_r restricted to those rows: the forward gathers A_r·E at h and t alone), which keeps it
seconds on the host.

Bars (as tests/test_gpu_config3.py):
  * logits: per edge, 1e-4 or 2x that edge's fp32-oracle drift (tests/parity.py); probabilities 1e-4;
    layer-3 rows max(1e-4, 2x the fp32 oracle's drift);
  * a full training step (forward + backward) is bitwise deterministic run to run (exact mode), and the
    split-fp16 GEMM mode agrees with it on every gradient to 2e-4 of max|g| at a non-saturating init;
  * the backward at this size against the oracle (tests/fullsize_grads.py): a sampled step with the FULL
    20M-entry adjacency and million-row node tables, exact and bf16x3, every gradient vs float64 autograd of
    the reference formulation (IDDGCN.py:146-174): 2e-4 of max|g| (mild init), max(2e-4, 2x fp32 drift)
    (reference init).
"""
import numpy as np
import pytest
import torch

from iddgcn_amd.engine import Engine, FlatParams
from iddgcn_amd.graph import get_adj_mats
from iddgcn_amd.utils import synthetic_graph
from oracle.ref_model import forward_detail, init_params
from oracle.ref_utils import get_adj_coo
from fullsize_grads import check_sampled_grads, grad_sample
from parity import assert_logits

pytestmark = pytest.mark.gpu
N, R, M, D = 1_000_000, 2, 20_000_000, 256


def mild_params(seed=1):
    rng = np.random.default_rng(seed)
    p = {"E": rng.standard_normal((N, D), dtype=np.float32) / np.float32(np.sqrt(D))}
    for l in (1, 2, 3):
        p[f"K{l}"] = rng.standard_normal((R, D, D)) / D
        p[f"S{l}"] = rng.standard_normal((D, D)) / np.sqrt(D)
        p[f"relw{l}"] = rng.uniform(-.05, .05, R)
        p[f"Wa{l}"] = rng.standard_normal((D, R)) / np.sqrt(D)
        p[f"ba{l}"] = rng.standard_normal(R) * 0.1
    p["rel"] = rng.standard_normal((R, D))
    return {k: v.astype(np.float32) for k, v in p.items()}


def restricted_coo(pos, triples, n, r):
    """get_adj_coo of the adjacency rows (objects) the scored triples touch: A_r·E restricted to the rows
    the forward gathers (IDDGCN.py:71-72), in the same sorted order per row."""
    need = np.unique(np.concatenate([triples[:, 0], triples[:, 2]]))
    return get_adj_coo(pos[np.isin(pos[:, 0], need)], n, r)


@pytest.fixture(scope="module")
def cfg4(cuda):
    pos, neg = synthetic_graph(N, R, M, seed=0)                 # bench.py's config-4 graph
    tri = np.concatenate([pos, neg])
    lab = np.concatenate([np.ones(len(pos), np.float32), np.zeros(len(neg), np.float32)])
    eng = Engine(N, R, D, cuda)
    adj = get_adj_mats(pos, N, R, device=cuda)
    ed = eng.edges(tri, lab)
    sample = np.sort(np.random.default_rng(0).choice(len(tri), 10_000, replace=False))
    coo = restricted_coo(pos, tri[sample], N, R)
    yield {"eng": eng, "adj": adj, "ed": ed, "tri": tri[sample], "sample": sample, "coo": coo, "pos": pos,
           "tri_all": tri, "lab_all": lab}
    eng.release()
    del eng, adj, ed
    torch.cuda.empty_cache()


@pytest.mark.parametrize("init,gemm", [("mild", "exact"), ("reference", "exact"), ("mild", "split"),
                                       ("reference", "bf16x3")])
def test_config4_forward_vs_oracle_sample(cfg4, init, gemm, cuda):
    params = mild_params() if init == "mild" else init_params(N, R, D, seed=89)
    eng, ed, sample = cfg4["eng"], cfg4["ed"], cfg4["sample"]
    eng.gemm = gemm
    P = FlatParams(N, R, D, cuda)
    P.load(params)
    p, s = eng.predict(P, cfg4["adj"], ed, logits=True)
    layers = eng.layer_outputs(ed, rows=sample)
    p64, s64, l64 = forward_detail(params, cfg4["tri"], cfg4["coo"], N, dtype=torch.float64)
    p32, s32, l32 = forward_detail(params, cfg4["tri"], cfg4["coo"], N, dtype=torch.float32)
    ps, ss = p.cpu().numpy()[sample], s.cpu().numpy()[sample]
    assert_logits(ss, s64, s32, f"config 4 {init} {gemm}")
    assert np.abs(ps - p64).max() <= 1e-4
    for side in (0, 1):
        ours = layers[2][side].cpu().numpy()
        err, drift = np.abs(ours - l64[2][side]).max(), np.abs(l32[2][side] - l64[2][side]).max()
        assert err <= max(1e-4, 2 * drift), f"layer 3 side {side}: {err:.2e} (fp32 drift {drift:.2e})"
    del P
    eng.release()


def test_config4_step_deterministic_and_modes_agree(cfg4, cuda):
    eng, ed, adj = cfg4["eng"], cfg4["ed"], cfg4["adj"]
    eng.release()                                   # the predict workspace: ~125 GB at T = 40M
    P = FlatParams(N, R, D, cuda)
    P.load(mild_params(2))
    out = {}
    for key, gemm in (("exact", "exact"), ("exact_again", "exact"), ("split", "split"), ("b3", "bf16x3")):
        eng.gemm = gemm
        G = FlatParams(N, R, D, cuda)
        loss, p = eng.loss_and_grads(P, G, adj, ed)
        out[key] = (float(loss.item()), p.cpu().numpy(), G.to_numpy())
        del G, p
    eng.release()
    a, b = out["exact"], out["exact_again"]
    assert np.isfinite(a[0]) and a[0] > 0
    assert a[0] == b[0] and np.array_equal(a[1], b[1])                       # bitwise run to run
    assert all(np.array_equal(a[2][k], b[2][k]) for k in a[2])
    for m in ("split", "b3"):
        c = out[m]
        assert abs(c[0] - a[0]) <= 1e-6 * abs(a[0]), m
        np.testing.assert_allclose(c[1], a[1], rtol=0, atol=1e-5)
        for k in a[2]:
            scale = np.abs(a[2][k]).max()
            assert np.all(np.isfinite(a[2][k])), k
            assert np.abs(c[2][k] - a[2][k]).max() <= 2e-4 * scale + 1e-30, (m, k)


@pytest.mark.parametrize("init", ["mild", "reference"])
def test_config4_step_grads_vs_oracle_sample(cfg4, init, cuda):
    cfg4["eng"].release()
    params = mild_params(3) if init == "mild" else init_params(N, R, D, seed=89)
    idx = grad_sample(cfg4["tri_all"], seed=4)
    check_sampled_grads(cfg4["eng"], cfg4["adj"], params, cfg4["pos"], cfg4["tri_all"][idx], cfg4["lab_all"][idx],
                        ("exact", "bf16x3"), cuda, saturating=init == "reference", what=f"config 4 {init}")
