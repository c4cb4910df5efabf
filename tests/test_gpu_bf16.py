"""The bf16-feature mode (BASELINE config 5: "bf16 features with MFMA XW"; perf only, no parity claim
to the fp32 reference): edge tables x^l / do^l stored as bf16, edge GEMMs on bf16 MFMA with fp32
accumulation and fp32 epilogues.

Kernel bars: each bf16 kernel against an fp64 torch reference of the same op evaluated on the SAME
bf16-rounded inputs — the only extra error allowed is the bf16 rounding of the output (2^-8 relative)
and the bf16 hi+lo representation of the weights (2^-16 relative; with IDDGCN_GEMM_BF16 the reference takes the
weights, and in the R = 8 forward the combine's node rows and coefficients, rounded to bf16 as the kernel does, so
the same bars hold): outputs within 6e-3 of max|ref|
for bf16-stored results, 1e-5 for fp32 results (TN partials, dP, logits of exact bf16 inputs).
Model bar: a bf16-mode training step against the fp32 engine on the same inputs — loss within 2e-2 relative,
probabilities within 2e-2, every gradient within 5e-2 of its max|g| (plus a floor of 1e-6 of the step's largest
gradient, for the saturated layer-3 gate parameters at R = 8).
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


def bf(x):
    return x.to(torch.bfloat16)


def rb(x):
    """x rounded to bf16 (RNE), as float64: an operand of the IDDGCN_GEMM_BF16 form."""
    return x.float().to(torch.bfloat16).double()


def maxrel(got, ref):
    return ((got.double() - ref).abs().max() / ref.abs().max()).item()


def tails(M, N, g):
    lengths = torch.randint(4, 60, (N,), generator=g)
    return torch.repeat_interleave(torch.arange(N), lengths)[:M]


@pytest.mark.parametrize("precision", ["exact", "bf16"])
@pytest.mark.parametrize("R", [1, 2, 8])
def test_rowgemm_bf16_forward_combine(R, precision, cuda):
    g = torch.Generator().manual_seed(R)
    N, M = 3000, 40_007
    A = bf(torch.rand(M, D, generator=g)).to(cuda)
    S = (torch.randn(D, D, generator=g, dtype=torch.float64) / 16).to(cuda)
    W = torch.rand(M, R, generator=g, dtype=torch.float64).to(cuda)
    P = torch.randn(R, N, D, generator=g, dtype=torch.float64).to(cuda)
    t = tails(M, N, g).to(cuda)
    ref = torch.sigmoid(A.double() @ S + sum(W[:, r:r + 1] * P[r][t] for r in range(R)))
    C = torch.empty(M, D, dtype=torch.bfloat16, device=cuda)
    ops.rowgemm(A, S.float(), C, coef=W.float(), V=P.float(), v_idx=t.int(), v_rel_stride=N * D, act=L.ACT_SIGMOID,
                precision=precision)
    if precision == "bf16":
        # IDDGCN_GEMM_BF16: the weights enter the MFMAs rounded to bf16; at R = 8 (fwd_gather8_bf16_kernel, the combine
        # on MFMAs) so do the node rows and coefficients, at R <= 2 the v3 kernel's combine stays fp32 on the VALU.  The
        # fp64 reference on the operands rounded the same way; the output's bf16 rounding (2^-8) + 1e-5 of max|ref|
        op = rb if R == 8 else (lambda x: x.float().double())
        ref = torch.sigmoid(A.double() @ rb(S) + sum(op(W)[:, r:r + 1] * op(P)[r][t] for r in range(R)))
        err = (C.double() - ref).abs()
        assert (err <= 2 ** -8 * ref.abs() + 1e-5 * ref.abs().max()).all(), err.max().item()
    else:
        assert maxrel(C, ref) <= 6e-3


@pytest.mark.parametrize("precision", ["exact", "bf16"])
@pytest.mark.parametrize("case", ["sorted", "short_runs", "unsorted", "tiny", "one_tile", "linear"])
def test_fwd_gather8_bf16(case, precision, cuda):
    """The R = 8 forward of the bf16-feature mode (fwd_gather8_bf16_kernel: x S and the gathered combine both on
    bf16 MFMAs, the tile's distinct V rows as the combine's k axis): element-wise within the bf16 rounding of the
    output (2^-8 relative) plus 1e-5 of max|ref| of the fp64 reference on the same bf16 inputs.  Tails sorted with
    runs of 4-60 and of 1-3 edges (up to 32 distinct V rows per tile), unsorted (the slots past the 8 staged ones),
    ragged and tiny M, and no activation.  precision "bf16" (IDDGCN_GEMM_BF16): the weights, node rows and
    coefficients enter the MFMAs rounded to bf16, so the fp64 reference takes them rounded the same way (the products
    of bf16 values are exact in fp32: the same bar)."""
    g = torch.Generator().manual_seed(hash(case) % 1000)
    N, M = 5000, {"tiny": 45, "one_tile": 32}.get(case, 60_013)
    if case == "short_runs":
        t = torch.repeat_interleave(torch.arange(N), torch.randint(1, 4, (N,), generator=g))[:M]
    elif case == "unsorted":
        t = torch.randint(0, N, (M,), generator=g)
    else:
        t = tails(M, N, g)
    M = len(t)
    A = bf(torch.rand(M, D, generator=g)).to(cuda)
    S = (torch.randn(D, D, generator=g, dtype=torch.float64) / 16).to(cuda)
    W = torch.rand(M, 8, generator=g, dtype=torch.float64).to(cuda)
    P = torch.randn(8, N, D, generator=g, dtype=torch.float64).to(cuda)
    t = t.to(cuda)
    op = rb if precision == "bf16" else (lambda x: x.float().double())
    z = A.double() @ op(S) + sum(op(W)[:, r:r + 1] * op(P)[r][t] for r in range(8))
    act = L.ACT_NONE if case == "linear" else L.ACT_SIGMOID
    ref = z if case == "linear" else torch.sigmoid(z)
    C = torch.full((M + 7, D), float("nan"), dtype=torch.bfloat16, device=cuda)
    ops.rowgemm(A, S.float(), C[:M], coef=W.float(), V=P.float(), v_idx=t.int(), v_rel_stride=N * D, act=act,
                precision=precision)
    err = (C[:M].double() - ref).abs()
    assert (err <= 2 ** -8 * ref.abs() + 1e-5 * ref.abs().max()).all(), err.max().item()
    assert C[M:].isnan().all()                 # nothing past row M is written


def test_fwd_gather8_unaligned_coef_takes_v3_path(cuda):
    """iddgcn_rowgemm_bf16 sends the R = 8 forward to fwd_gather8_bf16_kernel only with 16-B aligned A, C, coef and V
    (its DMAs move 16-B pieces); a coefficient table 4 B off alignment takes the v3 kernel: same bar against fp64,
    and within one bf16 ulp of the MFMA-combine result."""
    g = torch.Generator().manual_seed(12)
    N, M, R = 3000, 20_011, 8
    A = bf(torch.rand(M, D, generator=g)).to(cuda)
    S = (torch.randn(D, D, generator=g) / 16).to(cuda)
    W = torch.rand(M, R, generator=g).to(cuda)
    Wu = torch.empty(M * R + 1, device=cuda)[1:].view(M, R)
    Wu.copy_(W)
    P = torch.randn(R, N, D, generator=g).to(cuda)
    t = tails(M, N, g).to(cuda).int()
    ref = torch.sigmoid(A.double() @ S.double() + sum(W.double()[:, r:r + 1] * P.double()[r][t.long()] for r in range(R)))
    outs = []
    for coef in (W, Wu):
        C = torch.empty(M, D, dtype=torch.bfloat16, device=cuda)
        ops.rowgemm(A, S, C, coef=coef, V=P, v_idx=t, v_rel_stride=N * D, act=L.ACT_SIGMOID)
        err = (C.double() - ref).abs()
        assert (err <= 2 ** -8 * ref.abs() + 1e-5 * ref.abs().max()).all(), err.max().item()
        outs.append(C.double())
    assert (outs[0] - outs[1]).abs().max().item() <= 2 ** -8


def test_fwd_gather8_bf16_offsets_past_2e32(cuda):
    """fwd_gather8_bf16_kernel addresses relation r's node row as r·v_rel_stride + row·D in 64 bits: with N = 2.5M
    ((R-1)·N·D = 4.5e9 elements > 2^32) rows gathered from the top of the table, the same bar as above."""
    g = torch.Generator(device=cuda).manual_seed(31)
    R, N, M = 8, 2_500_000, 4096
    assert (R - 1) * N * D > 2 ** 32
    P = torch.randn(R, N, D, device=cuda, generator=g)
    t = (N - 1 - torch.sort(torch.randint(0, 600, (M,), device=cuda, generator=g), descending=True)[0]).int()
    A = bf(torch.rand(M, D, device=cuda, generator=g))
    S = torch.randn(D, D, device=cuda, generator=g) / 16
    W = torch.rand(M, R, device=cuda, generator=g)
    ref = torch.sigmoid(A.double() @ S.double() + sum(W[:, r:r + 1].double() * P[r][t.long()].double()
                                                      for r in range(R)))
    C = torch.empty(M, D, dtype=torch.bfloat16, device=cuda)
    ops.rowgemm(A, S, C, coef=W, V=P, v_idx=t, v_rel_stride=N * D, act=L.ACT_SIGMOID)
    del P
    torch.cuda.empty_cache()
    err = (C.double() - ref).abs()
    assert (err <= 2 ** -8 * ref.abs() + 1e-5 * ref.abs().max()).all(), err.max().item()


@pytest.mark.parametrize("precision", ["exact", "bf16"])
def test_rowgemm_bf16_backward_dsigmoid(precision, cuda):
    """The sigma' backward on bf16 tables; precision "bf16" (IDDGCN_GEMM_BF16): the weights rounded to bf16, so the
    fp64 reference takes them rounded too and every element must sit within the output's bf16 rounding (2^-8
    relative) plus 1e-5 of max|ref|."""
    g = torch.Generator().manual_seed(7)
    M = 30_001
    dO = bf(torch.randn(M, D, generator=g) * 1e-4).to(cuda)
    S = (torch.randn(D, D, generator=g, dtype=torch.float64) / 16).to(cuda)
    X = bf(torch.rand(M, D, generator=g)).to(cuda)
    ref = (dO.double() @ S.t()) * X.double() * (1 - X.double())
    C = torch.empty(M, D, dtype=torch.bfloat16, device=cuda)
    ops.rowgemm(dO, S.float(), C, b_trans=True, act=L.ACT_DSIGMOID, aux=X, precision=precision)
    assert maxrel(C, ref) <= 6e-3
    if precision == "bf16":
        ref_b = (dO.double() @ rb(S).t()) * X.double() * (1 - X.double())
        err = (C.double() - ref_b).abs()
        assert (err <= 2 ** -8 * ref_b.abs() + 1e-5 * ref_b.abs().max()).all(), err.max().item()
    Xi = X.clone()                     # in place over the sigma' operand, as the engine runs it
    ops.rowgemm(dO, S.float(), Xi, b_trans=True, act=L.ACT_DSIGMOID, aux=Xi, precision=precision)
    assert torch.equal(Xi, C)


@pytest.mark.parametrize("precision", ["exact", "bf16"])
def test_rowgemm_bf16_gathered_rows(precision, cuda):
    """bf16 A rows gathered by a_idx (the v3 kernel's two-rows-per-DMA staging takes each half-wave's row from its own
    index, round 5): random, repeated and ragged indices, plain and sigma' forms, within the output's bf16 rounding of
    the fp64 reference on the same bf16 inputs (the weights rounded too for precision "bf16")."""
    g = torch.Generator().manual_seed(21)
    Msrc, M = 5000, 20_003
    A = bf(torch.rand(Msrc, D, generator=g)).to(cuda)
    idx = torch.randint(0, Msrc, (M,), generator=g).int().to(cuda)
    idx[100:140] = 7                                   # a run of one repeated row
    S = (torch.randn(D, D, generator=g, dtype=torch.float64) / 16).to(cuda)
    Sd = rb(S) if precision == "bf16" else S.float().double()
    X = bf(torch.rand(M, D, generator=g)).to(cuda)
    Ag = A.double()[idx.long()]
    for act, aux, ref in ((L.ACT_NONE, None, Ag @ Sd), (L.ACT_SIGMOID, None, torch.sigmoid(Ag @ Sd)),
                          (L.ACT_DSIGMOID, X, (Ag @ Sd) * X.double() * (1 - X.double()))):
        C = torch.empty(M, D, dtype=torch.bfloat16, device=cuda)
        ops.rowgemm(A, S.float(), C, a_idx=idx, act=act, aux=aux, precision=precision)
        err = (C.double() - ref).abs()
        assert (err <= 2 ** -8 * ref.abs() + 1e-5 * ref.abs().max()).all(), (act, err.max().item())


def test_rowgemm_bf16_precision_refused_on_fp32_tables(cuda):
    """IDDGCN_GEMM_BF16 is a bf16-table form: iddgcn_rowgemm_f32 refuses it (IDDGCN_E_BAD_ARG, nothing launched)."""
    A = torch.rand(64, D, device=cuda)
    C = torch.empty(64, D, device=cuda)
    with pytest.raises(L.IddgcnError):
        ops.rowgemm(A, torch.randn(D, D, device=cuda), C, precision="bf16")


@pytest.mark.parametrize("M", [31, 5003, 300_017])
def test_gemm_tn_bf16(M, cuda):
    g = torch.Generator().manual_seed(M)
    A = bf(torch.randn(M, D, generator=g)).to(cuda)
    B = bf(torch.randn(M, D, generator=g) * 1e-3).to(cuda)
    ref = A.double().t() @ B.double()
    C = torch.empty(D, D, device=cuda)
    slab = torch.empty(ops.tn_blocks(M, D) * D * D, device=cuda)
    ops.gemm_tn(A, B, C, slab)
    assert maxrel(C, ref) <= 1e-5


@pytest.mark.parametrize("precision", ["exact", "bf16"])
@pytest.mark.parametrize("M", [0, 31, 5003, 300_017])
def test_sigma_tn_bf16_fused(M, precision, cuda):
    """iddgcn_sigma_tn_bf16 (ABI 11): dS = X^T dO and X = (dO S^T) X (1 - X) in place, in one pass — the bars of the two
    kernels it replaces (dS within 1e-5 of max|ref| of the fp64 product of the same bf16 tables; every dx element within
    the output's bf16 rounding plus 1e-5 of max|ref| of the fp64 reference with the weights as the kernel takes them:
    hi + lo, or rounded to bf16 for precision "bf16"), on full tiles, a ragged last tile, a table shorter than one
    tile and an empty one; dS is overwritten (a stale slab / output never leaks in)."""
    g = torch.Generator().manual_seed(M + 1)
    dO = bf(torch.randn(M, D, generator=g) * 1e-3).to(cuda)
    X = bf(torch.rand(M, D, generator=g)).to(cuda)
    S = (torch.randn(D, D, generator=g, dtype=torch.float64) / 16).to(cuda)
    Sd = rb(S) if precision == "bf16" else S.float().double()
    ref_S = X.double().t() @ dO.double()
    ref_x = (dO.double() @ Sd.t()) * X.double() * (1 - X.double())
    slab = torch.full((ops.sigma_tn_slab_floats(M),), float("nan"), device=cuda)
    dS = torch.full((D, D), float("nan"), device=cuda)
    Xi = X.clone()
    ops.sigma_tn(dO, Xi, S.float(), dS, slab, precision=precision)
    torch.cuda.synchronize()
    if M == 0:
        assert torch.equal(dS, torch.zeros_like(dS))
        return
    assert (dS.double() - ref_S).abs().max().item() <= 1e-5 * ref_S.abs().max().item()
    err = (Xi.double() - ref_x).abs()
    assert (err <= 2 ** -8 * ref_x.abs() + 1e-5 * ref_x.abs().max()).all(), err.max().item()
    # the same dx as the sigma' kernel it replaces, up to the fp32 accumulation order (one bf16 rounding step apart
    # at most)
    C = torch.empty(M, D, dtype=torch.bfloat16, device=cuda)
    ops.rowgemm(dO, S.float(), C, b_trans=True, act=L.ACT_DSIGMOID, aux=X, precision=precision)
    diff = (Xi.double() - C.double()).abs()
    assert (diff <= 2 ** -7 * C.double().abs() + 1e-6 * ref_x.abs().max()).all(), diff.max().item()


@pytest.mark.parametrize("R", [2, 8])
def test_combine_tail_seg_distmult_bf16(R, cuda):
    g = torch.Generator().manual_seed(11 * R)
    N, M = 2000, 50_000
    t = tails(M, N, g).to(cuda).int()
    Y = torch.randn(N, D, generator=g).to(cuda)
    W = torch.rand(M, R, generator=g).to(cuda)
    P = torch.randn(R, N, D, generator=g).to(cuda)
    out = torch.empty(M, D, dtype=torch.bfloat16, device=cuda)
    ops.combine(Y, W, P, out, y_idx=t, v_idx=t)
    tl = t.long()
    ref = torch.sigmoid(Y.double()[tl] + sum(W.double()[:, r:r + 1] * P.double()[r][tl] for r in range(R)))
    assert maxrel(out, ref) <= 6e-3
    # tail-side segmented reduction over bf16 rows == the fp32 kernel on the same (widened) rows: bitwise for the
    # VALU form (R < 8); R = 8 runs the MFMA form (tail_seg_mfma8_kernel: exact three-piece operands, fp32 sums in
    # another order), within 1e-5 of max|ref| of it
    tptr = torch.searchsorted(t, torch.arange(N + 1, device=cuda, dtype=torch.int32)).int()
    dP, dWe = torch.empty(R, N, D, device=cuda), torch.empty(M, R, device=cuda)
    ops.tail_seg_reduce(tptr, None, W, out, P, dP, dWe)
    dP32, dWe32 = torch.empty_like(dP), torch.empty_like(dWe)
    ops.tail_seg_reduce(tptr, None, W, out.float(), P, dP32, dWe32)
    if R < 8:
        assert torch.equal(dP, dP32) and torch.equal(dWe, dWe32)
    else:
        assert maxrel(dP, dP32.double()) <= 1e-5 and maxrel(dWe, dWe32.double()) <= 1e-5
    # DistMult scores of bf16 tails == the fp32 kernel on the widened rows
    h = torch.randint(0, N, (M,), generator=g).int().to(cuda)
    r = torch.randint(0, R, (M,), generator=g).int().to(cuda)
    rel = torch.randn(R, D, generator=g).to(cuda)
    Xh = torch.rand(N, D, generator=g).to(cuda)
    p, s = torch.empty(M, device=cuda), torch.empty(M, device=cuda)
    ops.distmult_bce(Xh, h, out, r, rel, p_out=p, s_out=s)
    p32, s32 = torch.empty_like(p), torch.empty_like(s)
    ops.distmult_bce(Xh, h, out.float(), r, rel, p_out=p32, s_out=s32)
    assert torch.equal(s, s32) and torch.equal(p, p32)


@pytest.mark.parametrize("edge_mfma", ["hilo", "bf16"])
@pytest.mark.parametrize("R", [2, 8])
def test_bf16_mode_step_tracks_fp32(R, edge_mfma, cuda):
    N = 1500
    pos, neg = synthetic_graph(N, R, 16000, seed=40 + R)
    tri = np.concatenate([pos, neg])
    lab = np.concatenate([np.ones(len(pos)), np.zeros(len(neg))])
    rng = np.random.default_rng(R)
    params = {"E": rng.standard_normal((N, D)) / np.sqrt(D), "rel": rng.standard_normal((R, D))}
    for l in (1, 2, 3):
        params.update({f"K{l}": rng.standard_normal((R, D, D)) / D, f"S{l}": rng.standard_normal((D, D)) / np.sqrt(D),
                       f"Wa{l}": rng.standard_normal((D, R)) / np.sqrt(D), f"ba{l}": rng.standard_normal(R) * 0.1})
    out = {}
    for feat in ("f32", "bf16"):
        eng = Engine(N, R, D, cuda, features=feat, edge_mfma=edge_mfma if feat == "bf16" else "hilo")
        P, G = FlatParams(N, R, D, cuda), FlatParams(N, R, D, cuda)
        P.load(params)
        adj = eng.adjacency(get_adj_mats(pos, N, R))
        loss, p = eng.loss_and_grads(P, G, adj, eng.edges(tri, lab))
        out[feat] = (float(loss.item()), p.cpu().numpy(), G.to_numpy())
    (l32, p32, g32), (lb, pb, gb) = out["f32"], out["bf16"]
    assert abs(lb - l32) <= 2e-2 * l32
    assert np.abs(pb - p32).max() <= 2e-2
    # floor: 1e-6 of the step's largest gradient.  At R = 8 the layer-3 sigmoid saturates on nearly every row of this
    # graph, so W_alpha^3 / b_alpha^3 get gradients at the rounding-noise floor (0 to 1e-13 against 8e-5 for S3, and
    # either mode may land on either side of a saturation boundary); a relative bar on those compares noise.
    floor = 1e-6 * max(np.abs(v).max() for v in g32.values())
    for k, v in g32.items():
        assert np.all(np.isfinite(gb[k])), k
        assert np.abs(gb[k] - v).max() <= 5e-2 * np.abs(v).max() + floor, k


@pytest.mark.parametrize("case", ["uniform", "hub", "sparse", "empty", "tiny", "long"])
@pytest.mark.parametrize("dsum", [False, True])
def test_tail_seg_mfma8_bf16(case, dsum, cuda):
    """The R = 8 bf16 tail reduction on MFMAs (tail_seg_mfma8_kernel, config 5's form: per-edge W, bf16 do rows) against
    float64 index_add references on the same bf16 rows: dP, dWedge and dsum within 1e-5 of max|ref| (the operands
    W and P enter as exact three-piece bf16 splits, so only the fp32 summation order differs); run twice, bitwise
    equal.  Cases: runs of tails without edges, a hub tail with a third of the edges, almost every tail without
    edges, tiny graphs (chunks of 32 edges padded), and segments of 1-200 edges (several chunks, partial last)."""
    g = torch.Generator().manual_seed(len(case) * 7 + dsum)
    R = 8
    N = {"tiny": 5, "empty": 300, "long": 400}.get(case, 1000 + 7)
    T = {"tiny": 37, "empty": 3, "sparse": 60}.get(case, 30_000)
    if case == "long":
        lengths = torch.randint(1, 200, (N,), generator=g)
        t = torch.repeat_interleave(torch.arange(N), lengths)
        T = len(t)
    else:
        t = torch.randint(0, N, (T,), generator=g)
        if case == "hub":
            t[: T // 3] = 517
        if case == "uniform":
            t[(t >= 100) & (t < 140)] = 99
        t = torch.sort(t).values
    tptr = torch.searchsorted(t, torch.arange(N + 1), right=False).to(torch.int32).to(cuda)
    W = torch.rand(T, R, generator=g).to(cuda)
    P = torch.randn(R, N, D, generator=g).to(cuda)
    dO = bf(torch.randn(T, D, generator=g)).to(cuda)
    tc = t.to(cuda)
    outs = []
    for _ in range(2):
        dP, dWe = torch.full((R, N, D), 7.0, device=cuda), torch.full((T, R), 7.0, device=cuda)
        ds = torch.full((N, D), 7.0, device=cuda) if dsum else None
        ops.tail_seg_reduce(tptr, None, W, dO, P, dP, dWe, dsum=ds)
        outs.append([dP, dWe] + ([ds] if dsum else []))
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    dP, dWe = outs[0][0], outs[0][1]
    d64, W64, P64 = dO.double(), W.double(), P.double()
    for r in range(R):
        ref = torch.zeros(N, D, dtype=torch.float64, device=cuda).index_add_(0, tc, W64[:, r:r + 1] * d64)
        assert (dP[r].double() - ref).abs().max().item() <= 1e-5 * max(ref.abs().max().item(), 1e-30)
        if T:
            refw = (d64 * P64[r][tc]).sum(-1)
            assert (dWe[:, r].double() - refw).abs().max().item() <= 1e-5 * refw.abs().max().item()
    if dsum:
        ref = torch.zeros(N, D, dtype=torch.float64, device=cuda).index_add_(0, tc, d64)
        assert (outs[0][2].double() - ref).abs().max().item() <= 1e-5 * max(ref.abs().max().item(), 1e-30)


@pytest.mark.parametrize("dsum", [False, True])
def test_tail_seg_reduce_head_fused_equals_two_calls(dsum, cuda):
    """iddgcn_tail_seg_reduce_head_bf16 (ABI 9: the R = 8 tail reduction that adds the head chain's node terms
    Wn[n] head_dO[n] to dP and head_dO[n] to dsum before its store, and forms dwh[n] = <head_dO[n], P_r[n]>) followed
    by head_dz equals tail_seg_reduce + head_bwd_node: dP, dsum, dWedge, dz within 1e-6 of max|ref| (the same terms in
    other fp32 orders); dwh within 1e-6 of float64."""
    g = torch.Generator().manual_seed(5 + dsum)
    R, N, M = 8, 600, 20_000
    t = tails(M, N, g).to(cuda).int()
    M = len(t)
    tptr = torch.searchsorted(t, torch.arange(N + 1, device=cuda, dtype=torch.int32)).int()
    W = torch.rand(M, R, generator=g).to(cuda)
    P = torch.randn(R, N, D, generator=g).to(cuda)
    dO = bf(torch.randn(M, D, generator=g)).to(cuda)
    hd = torch.randn(N, D, generator=g).to(cuda)
    Wn = torch.rand(N, R, generator=g).to(cuda)
    Ssm = torch.rand(N, R, generator=g).to(cuda)
    h = torch.randint(0, N, (M,), generator=g).to(cuda)
    hperm = torch.argsort(h, stable=True).int()
    hptr = torch.searchsorted(h[hperm.long()], torch.arange(N + 1, device=cuda)).int()
    out = []
    for fused in (False, True):
        dP, dWe = torch.empty(R, N, D, device=cuda), torch.empty(M, R, device=cuda)
        ds = torch.empty(N, D, device=cuda) if dsum else None
        dz = torch.empty(N, R, device=cuda)
        if fused:
            dwh = torch.empty(N, R, device=cuda)
            ops.tail_seg_reduce_head(tptr, W, dO, P, dP, dWe, hd, Wn, dwh, dsum=ds)
            ops.head_dz(Ssm, Wn, hptr, hperm, dWe, dwh, dz)
            ref = torch.einsum("nd,rnd->nr", hd.double(), P.double())
            assert maxrel(dwh, ref) <= 1e-6
        else:
            ops.tail_seg_reduce(tptr, None, W, dO, P, dP, dWe, dsum=ds)
            ops.head_bwd_node(hd, P, Ssm, Wn, dP, dz, hseg_ptr=hptr, hperm=hperm, dWedge=dWe, dsum=ds)
        out.append([dP, dWe, dz] + ([ds] if dsum else []))
    for a, b in zip(*out):
        assert maxrel(b, a.double()) <= 1e-6
