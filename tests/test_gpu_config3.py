"""BASELINE config 3 at FULL size on the GPU (100k nodes, 2 relations, 2M edges, D=256, 4M scored
edges): the shapes that only exist at this scale — many 32-row tiles per persistent workgroup, long
tail / head segments, edge tables of 4.1 GB (element offsets past 2^30) — checked against the float64
oracle (oracle/ref_model.py, IDDGCN.py:60-178) on a 10k scored-edge sample, in both GEMM operand modes.

Bars (as tests/test_gpu_model.py):
  * logits: per edge, 1e-4 or 2x that edge's fp32-oracle drift (tests/parity.py);
  * probabilities 1e-4; layer-3 outputs x_h^3, x_t^3 max(1e-4, 2x fp32 drift);
  * a training step is bitwise deterministic; the split-fp16 and exact-f32 GEMM modes agree on every
    gradient to 2e-4 of its max |g| at a non-saturating init (N(0, 1/D)-scaled weights);
  * the backward at this size against the oracle (tests/fullsize_grads.py): every gradient of a sampled step
    (random scored edges + complete tail / head segments) run with the FULL adjacency and node tables, exact
    and bf16x3, vs float64 autograd of the reference formulation (IDDGCN.py:146-174): 2e-4 of max|g| at the
    mild init, max(2e-4, 2x the fp32 oracle's drift) at the reference init.
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
N, R, M, D = 100_000, 2, 2_000_000, 256


def mild_params(seed=1):
    rng = np.random.default_rng(seed)
    p = {"E": rng.standard_normal((N, D)) / np.sqrt(D)}
    for l in (1, 2, 3):
        p[f"K{l}"] = rng.standard_normal((R, D, D)) / D
        p[f"S{l}"] = rng.standard_normal((D, D)) / np.sqrt(D)
        p[f"relw{l}"] = rng.uniform(-.05, .05, R)
        p[f"Wa{l}"] = rng.standard_normal((D, R)) / np.sqrt(D)
        p[f"ba{l}"] = rng.standard_normal(R) * 0.1
    p["rel"] = rng.standard_normal((R, D))
    return {k: v.astype(np.float32) for k, v in p.items()}


@pytest.fixture(scope="module")
def cfg3(cuda):
    pos, neg = synthetic_graph(N, R, M, seed=0)                 # bench.py's config-3 graph
    tri = np.concatenate([pos, neg])
    lab = np.concatenate([np.ones(len(pos), np.float32), np.zeros(len(neg), np.float32)])
    eng = Engine(N, R, D, cuda)
    adj = get_adj_mats(pos, N, R, device=cuda)
    ed = eng.edges(tri, lab)
    rng = np.random.default_rng(0)
    sample = np.sort(rng.choice(len(tri), 10_000, replace=False))
    coo = get_adj_coo(pos, N, R)
    yield {"eng": eng, "adj": adj, "ed": ed, "tri": tri, "sample": sample, "coo": coo, "pos": pos, "lab": lab}
    del eng, adj, ed
    torch.cuda.empty_cache()


@pytest.mark.parametrize("init", ["mild", "reference"])
@pytest.mark.parametrize("gemm", ["split", "exact", "bf16x3"])
def test_config3_forward_vs_oracle_sample(cfg3, init, gemm, cuda):
    params = mild_params() if init == "mild" else init_params(N, R, D, seed=89)
    eng, ed, sample = cfg3["eng"], cfg3["ed"], cfg3["sample"]
    eng.gemm = gemm
    P = FlatParams(N, R, D, cuda)
    P.load(params)
    p, s = eng.predict(P, cfg3["adj"], ed, logits=True)
    layers = eng.layer_outputs(ed, rows=sample)
    p64, s64, l64 = forward_detail(params, cfg3["tri"][sample], cfg3["coo"], N, dtype=torch.float64)
    p32, s32, l32 = forward_detail(params, cfg3["tri"][sample], cfg3["coo"], N, dtype=torch.float32)
    ps, ss = p.cpu().numpy()[sample], s.cpu().numpy()[sample]
    assert_logits(ss, s64, s32, f"config 3 {init} {gemm}")
    assert np.abs(ps - p64).max() <= 1e-4
    for side in (0, 1):
        ours = layers[2][side].cpu().numpy()
        err, drift = np.abs(ours - l64[2][side]).max(), np.abs(l32[2][side] - l64[2][side]).max()
        assert err <= max(1e-4, 2 * drift), f"layer 3 side {side}: {err:.2e} (fp32 drift {drift:.2e})"


def test_config3_step_deterministic_and_modes_agree(cfg3, cuda):
    eng, ed, adj = cfg3["eng"], cfg3["ed"], cfg3["adj"]
    params = mild_params(2)
    P = FlatParams(N, R, D, cuda)
    P.load(params)
    out = {}
    for key, gemm in (("split", "split"), ("split_again", "split"), ("exact", "exact"), ("b3", "bf16x3"),
                      ("b3_again", "bf16x3")):
        eng.gemm = gemm
        G = FlatParams(N, R, D, cuda)
        loss, p = eng.loss_and_grads(P, G, adj, ed)
        out[key] = (float(loss.item()), p.cpu().numpy(), G.to_numpy())
        del G
    c = out["exact"]
    for m in ("split", "b3"):
        a, b = out[m], out[m + "_again"]
        assert a[0] == b[0] and np.array_equal(a[1], b[1]), m                    # bitwise run to run
        assert all(np.array_equal(a[2][k], b[2][k]) for k in a[2]), m
        assert abs(a[0] - c[0]) <= 1e-6 * abs(c[0]), m
        np.testing.assert_allclose(a[1], c[1], rtol=0, atol=1e-5)
        for k in a[2]:
            scale = np.abs(c[2][k]).max()
            assert np.all(np.isfinite(a[2][k])), (m, k)
            assert np.abs(a[2][k] - c[2][k]).max() <= 2e-4 * scale + 1e-30, (m, k)


@pytest.mark.parametrize("init", ["mild", "reference"])
def test_config3_step_grads_vs_oracle_sample(cfg3, init, cuda):
    params = mild_params(3) if init == "mild" else init_params(N, R, D, seed=89)
    idx = grad_sample(cfg3["tri"], seed=3)
    check_sampled_grads(cfg3["eng"], cfg3["adj"], params, cfg3["pos"], cfg3["tri"][idx], cfg3["lab"][idx],
                        ("exact", "bf16x3"), cuda, saturating=init == "reference", what=f"config 3 {init}")
