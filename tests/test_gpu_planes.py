"""Pre-split ("planes") edge tables, include/iddgcn.h IDDGCN_PLANES_*: a D = 256 row of values in [0, 1]
stored as 8 column blocks of [hi f16[32] | lo f16[32]] with x * 2^15 = hi + lo.  The layer-1 combine and the layer-2
forward GEMM write x^1, x^2 this way; the layer-2/3 forward GEMMs (A), the dS TN GEMMs (A) and the sigma'
backward (aux) read them without converting.  Checks:
  * the producers' planes equal the torch encoding of their fp32 outputs (|decode - fp32| <= 2^-24);
  * each consumer on a planes table matches the same kernel on the decoded fp32 table (bitwise where the
    arithmetic is the same, else within 1e-6 of max|C|) and the fp64 reference (split-mode bars);
  * invalid flag combinations are refused;
  * a full D = 256 step with planes on vs off (Engine(planes=False)).
"""
import numpy as np
import pytest
import torch

from iddgcn_amd import _lib as L
from iddgcn_amd import ops
from iddgcn_amd.engine import Engine, FlatParams
from iddgcn_amd.graph import get_adj_mats
from iddgcn_amd.utils import synthetic_graph

pytestmark = pytest.mark.gpu
D = 256


SPLIT = dict(precision="split")      # the planes forms exist in the split-fp16 GEMM mode only


def to_planes(x):
    """torch restatement of the planes encoding: 8 column blocks of [hi f16[32] | lo f16[32]] per row,
    x * 2^15 = hi + lo (round-to-nearest-even fp16 casts)."""
    xs = x.float() * 2.0 ** 15
    hi = xs.half()
    lo = (xs - hi.float()).half()
    M = x.shape[0]
    return torch.stack([hi.view(M, 8, 32), lo.view(M, 8, 32)], 2).reshape(M, 512).contiguous().view(torch.float32)


def unit_rows(M, gen, dev, lo=0.0):
    """Rows of values in [lo, 1) with the max in [0.5, 1) (sigmoid-like)."""
    x = torch.rand(M, D, generator=gen) * (1.0 - lo) + lo
    x[:, 0] = 0.5 + 0.49 * torch.rand(M, generator=gen)
    return x.to(dev)


def test_planes_roundtrip(cuda):
    g = torch.Generator().manual_seed(0)
    x = unit_rows(1000, g, cuda)
    x[3] = 0.0
    x[4, :8] = torch.tensor([1.0, 2.0 ** -20, 2.0 ** -28, 1e-30, 0.999999, 0.5, 0.25, 3e-5])
    d = ops.planes_to_f32(to_planes(x))
    assert (d - x).abs().max().item() <= 2.0 ** -24


@pytest.mark.parametrize("R", [1, 2])
def test_combine_planes_out(R, cuda):
    g = torch.Generator().manual_seed(R)
    N, M = 3000, 20011
    Y = torch.randn(N, D, generator=g).to(cuda)
    V = torch.randn(R, N, D, generator=g).to(cuda)
    idx = torch.sort(torch.randint(0, N, (M,), generator=g)).values.int().to(cuda)
    coef = torch.rand(M, R, generator=g).to(cuda)
    o32 = torch.empty(M, D, device=cuda)
    opl = torch.empty(M, D, device=cuda)
    ops.combine(Y, coef, V, o32, y_idx=idx, v_idx=idx)
    ops.combine(Y, coef, V, opl, y_idx=idx, v_idx=idx, planes_out=True)
    assert torch.equal(opl, to_planes(o32))
    assert (ops.planes_to_f32(opl) - o32).abs().max().item() <= 2.0 ** -24


def _fwd_inputs(M, N, R, g, dev):
    S = (torch.randn(D, D, generator=g) / 16).to(dev)
    W = torch.rand(M, R, generator=g).to(dev)
    P = torch.randn(R, N, D, generator=g).to(dev)
    t = torch.sort(torch.randint(0, N, (M,), generator=g)).values.int().to(dev)
    return S, W, P, t


@pytest.mark.parametrize("M", [32, 1000, 40009])
def test_rowgemm_planes_a_and_c(M, cuda):
    """Gathered forward x^{l+1} = sigmoid(x^l S + sum_r w_r P_r[t]) with A planes (and C planes)."""
    g = torch.Generator().manual_seed(M)
    N, R = 5000, 2
    x = unit_rows(M, g, cuda)
    xp = to_planes(x)
    xd = ops.planes_to_f32(xp)
    S, W, P, t = _fwd_inputs(M, N, R, g, cuda)
    kw = dict(coef=W, V=P, v_idx=t, v_rel_stride=N * D, act=L.ACT_SIGMOID, **SPLIT)
    c32, cpa, cpl = (torch.empty(M, D, device=cuda) for _ in range(3))
    ops.rowgemm(xd, S, c32, **kw)
    ops.rowgemm(xp, S, cpa, planes=L.PLANES_A, **kw)
    ops.rowgemm(xp, S, cpl, planes=L.PLANES_A | L.PLANES_C, **kw)
    assert ops.rowgemm_kernel_id(xp, S, cpl, planes=L.PLANES_A | L.PLANES_C, **kw) == 3322
    # A planes vs the per-row split of the same values: the same hi / lo except at re-split ties
    assert (cpa - c32).abs().max().item() <= 1e-6
    # C planes: the planes encoding of the same fp32 epilogue values
    assert (ops.planes_to_f32(cpl) - cpa).abs().max().item() <= 2.0 ** -24
    pre = xd.double() @ S.double() + (W.double()[:, :, None] * P.double()[:, t.long()].permute(1, 0, 2)).sum(1)
    ref = torch.sigmoid(pre)
    assert (cpa.double() - ref).abs().max().item() <= 2e-6


@pytest.mark.parametrize("inplace", [False, True])
def test_rowgemm_planes_aux(inplace, cuda):
    """sigma' backward do^{l} = (do^{l+1} S^T) * x(1-x) with x^l a planes table (written over it)."""
    g = torch.Generator().manual_seed(7)
    M = 30017
    x = unit_rows(M, g, cuda, lo=0.0)
    xp = to_planes(x)
    xd = ops.planes_to_f32(xp)
    do = (torch.randn(M, D, generator=g) * 1e-3).to(cuda)
    S = (torch.randn(D, D, generator=g) / 16).to(cuda)
    c32 = torch.empty(M, D, device=cuda)
    cpl = xp.clone() if inplace else torch.empty(M, D, device=cuda)
    ops.rowgemm(do, S, c32, b_trans=True, act=L.ACT_DSIGMOID, aux=xd, **SPLIT)
    ops.rowgemm(do, S, cpl, b_trans=True, act=L.ACT_DSIGMOID, aux=xp.clone() if not inplace else cpl,
                planes=L.PLANES_AUX, **SPLIT)
    assert torch.equal(cpl, c32)          # sigma' from the same fp32 values, same GEMM


@pytest.mark.parametrize("M", [31, 4096, 250013])
def test_gemm_tn_planes_a(M, cuda):
    """dS = x^T do with x a planes table vs the fp32 TN on the decoded values and vs fp64."""
    g = torch.Generator().manual_seed(M)
    x = unit_rows(M, g, cuda)
    xp = to_planes(x)
    xd = ops.planes_to_f32(xp)
    do = (torch.randn(M, D, generator=g) * 1e-3).to(cuda)
    slab = torch.empty(ops.tn_blocks(M, D) * D * D, device=cuda)
    c32, cpl = torch.empty(D, D, device=cuda), torch.empty(D, D, device=cuda)
    ops.gemm_tn(xd, do, c32, slab, **SPLIT)
    ops.gemm_tn(xp, do, cpl, slab, a_planes=True, **SPLIT)
    ref = xd.double().t() @ do.double()
    scale = ref.abs().max().item()
    assert (cpl.double() - c32.double()).abs().max().item() <= 1e-6 * scale
    assert (cpl.double() - ref).abs().max().item() <= 2e-6 * scale


def test_planes_flag_checks(cuda):
    M, N, R = 64, 100, 2
    g = torch.Generator().manual_seed(1)
    x = unit_rows(M, g, cuda)
    S, W, P, t = _fwd_inputs(M, N, R, g, cuda)
    C = torch.empty(M, D, device=cuda)
    with pytest.raises(L.IddgcnError):         # planes C needs the sigmoid epilogue
        ops.rowgemm(x, S, C, coef=W, V=P, v_idx=t, v_rel_stride=N * D, planes=L.PLANES_C, **SPLIT)
    with pytest.raises(L.IddgcnError):         # planes aux needs DSIGMOID
        ops.rowgemm(x, S, C, planes=L.PLANES_AUX, **SPLIT)
    with pytest.raises(L.IddgcnError):         # unknown bit
        ops.rowgemm(x, S, C, planes=8, **SPLIT)
    with pytest.raises(L.IddgcnError):         # exact mode has no planes form
        ops.rowgemm(x, S, C, planes=L.PLANES_A, precision="exact")
    with pytest.raises(L.IddgcnError):         # nor has the exact TN
        ops.gemm_tn(x, x, torch.empty(D, D, device=cuda), torch.empty(ops.tn_blocks(M, D) * D * D, device=cuda),
                    a_planes=True, precision="exact")


def test_engine_step_planes_on_off(cuda):
    """Full D = 256 training step: x^1, x^2 pre-split (default) vs fp32 tables (planes=False)."""
    N, R = 3000, 2
    pos, neg = synthetic_graph(N, R, 12000, seed=21)
    rng = np.random.default_rng(3)
    params = {"E": rng.standard_normal((N, D)) / 8}
    for l in (1, 2, 3):
        params.update({f"K{l}": rng.standard_normal((R, D, D)) / D, f"S{l}": rng.standard_normal((D, D)) / 8,
                       f"relw{l}": np.zeros(R), f"Wa{l}": rng.standard_normal((D, R)) / 8, f"ba{l}": np.zeros(R)})
    params["rel"] = rng.standard_normal((R, D)) / 4
    params = {k: v.astype(np.float32) for k, v in params.items()}
    tri = np.concatenate([pos, neg])
    lab = np.concatenate([np.ones(len(pos)), np.zeros(len(neg))])
    out = []
    for planes in (True, False):
        eng = Engine(N, R, D, cuda, gemm="split", planes=planes)
        assert eng.use_planes == planes
        P, G = FlatParams(N, R, D, cuda), FlatParams(N, R, D, cuda)
        P.load(params)
        adj = eng.adjacency(get_adj_mats(pos, N, R))
        ed = eng.edges(tri, lab)
        loss, p, s = eng.loss_and_grads(P, G, adj, ed, logits=True)
        eng.predict(P, adj, ed)
        layers = eng.layer_outputs(ed, rows=np.arange(0, len(tri), 7))
        out.append((loss.item(), s.cpu().numpy(), G.to_numpy(), [(a.cpu().numpy(), b.cpu().numpy()) for a, b in layers]))
    (l1, s1, g1, y1), (l0, s0, g0, y0) = out
    assert abs(l1 - l0) <= 1e-6 * abs(l0)
    assert np.abs(s1 - s0).max() <= 1e-5
    for k in g0:
        assert np.abs(g1[k] - g0[k]).max() <= 1e-4 * np.abs(g0[k]).max() + 1e-30, k
    for (h1, t1), (h0, t0) in zip(y1, y0):
        assert np.array_equal(h1, h0)
        assert np.abs(t1 - t0).max() <= 1e-6
