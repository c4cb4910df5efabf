"""Per-kernel numerics on the GPU, each against a plain torch reference of the same op.

Tolerances: fp32 kernels vs an fp64 torch reference, |err| <= 2e-5 * (1 + |ref|)
scaled by the reduction length where sums are long.  Index/permutation work is exact.
"""
import numpy as np
import pytest
import torch

from iddgcn_amd import _lib as L
from iddgcn_amd import ops

pytestmark = pytest.mark.gpu
DIMS = [32, 64, 128, 256]


def rnd(*s, dev, scale=1.0, gen=None):
    return (torch.randn(*s, generator=gen, dtype=torch.float64) * scale).to(dev)


def close(got, ref, tol):
    got = got.double()
    err = (got - ref).abs().max().item()
    lim = tol * (1.0 + ref.abs().max().item())
    assert err <= lim, f"max err {err} > {lim}"


@pytest.mark.parametrize("D", DIMS)
def test_spmm_csr(D, cuda):
    g = torch.Generator().manual_seed(D)
    N, R, nnz = 517, 3, 4000
    rows = torch.randint(0, N, (R, nnz), generator=g)
    cols = torch.randint(0, N, (R, nnz), generator=g)
    X = rnd(N, D, dev=cuda, gen=g)
    ptrs, colsl, ref = [], [], torch.zeros(R, N, D, dtype=torch.float64, device=cuda)
    off = 0
    for r in range(R):
        key = torch.unique(rows[r] * N + cols[r])
        rr, cc = key // N, key % N
        ptr = torch.zeros(N + 1, dtype=torch.int64)
        ptr[1:] = torch.cumsum(torch.bincount(rr, minlength=N), 0)
        ptrs.append(ptr + off)
        colsl.append(cc)
        off += cc.numel()
        ref[r].index_add_(0, rr.to(cuda), X[cc.to(cuda)])
    ptr = torch.cat(ptrs).to(torch.int32).to(cuda)
    col = torch.cat(colsl).to(torch.int32).to(cuda)
    Y = torch.empty(R, N, D, device=cuda)
    ops.spmm_csr(ptr, col, None, X.float(), Y, R, N)
    close(Y, ref, 1e-5)
    vals = torch.rand(off, generator=g).to(cuda)
    Y2 = Y.clone()
    ops.spmm_csr(ptr, col, vals, X.float(), Y2, R, N, accumulate=True)
    ref2 = ref.clone()
    start = 0
    for r in range(R):
        n = colsl[r].numel()
        rr = torch.repeat_interleave(torch.arange(N), torch.diff(ptrs[r]))
        ref2[r].index_add_(0, rr.to(cuda), X[colsl[r].to(cuda)] * vals[start:start + n, None].double())
        start += n
    close(Y2, ref2, 1e-5)


@pytest.mark.parametrize("D", DIMS)
def test_sddmm_csr(D, cuda):
    """out[k] = <G[s][row_k], X[col_k]> over a batched CSR with empty rows and one long row."""
    g = torch.Generator().manual_seed(100 + D)
    N, R = 301, 3
    ptrs, cols, rows_all, off = [], [], [], 0
    for r in range(R):
        rows = torch.randint(0, N, (2000,), generator=g)
        rows[:300] = 5                                  # one long row
        rows = rows[rows % 7 != 3]                      # some empty rows
        c = torch.randint(0, N, (rows.numel(),), generator=g)
        key = torch.unique(rows * N + c)
        rr, cc = key // N, key % N
        ptr = torch.zeros(N + 1, dtype=torch.int64)
        ptr[1:] = torch.cumsum(torch.bincount(rr, minlength=N), 0)
        ptrs.append(ptr + off)
        cols.append(cc)
        rows_all.append(rr + r * N)
        off += cc.numel()
    ptr = torch.cat(ptrs).to(torch.int32).to(cuda)
    col = torch.cat(cols).to(torch.int32).to(cuda)
    Gm, Xm = rnd(R, N, D, dev=cuda, gen=g), rnd(N, D, dev=cuda, gen=g)
    out = torch.full((off,), 7.0, device=cuda)
    ops.sddmm_csr(ptr, col, Gm.float(), Xm.float(), out, R, N)
    rows = torch.cat(rows_all).to(cuda)
    ref = (Gm.view(R * N, D)[rows] * Xm[torch.cat(cols).to(cuda)]).sum(-1)
    close(out, ref, 1e-5 * np.sqrt(D))


@pytest.mark.parametrize("D", DIMS)
@pytest.mark.parametrize("trans", [False, True])
def test_rowgemm_plain(D, trans, cuda):
    g = torch.Generator().manual_seed(7 * D + trans)
    M = 1000 + D // 32        # not a multiple of any tile height
    A, B = rnd(M, D, dev=cuda, gen=g), rnd(D, D, dev=cuda, gen=g)
    C = torch.empty(M, D, device=cuda)
    ops.rowgemm(A.float(), B.float(), C, b_trans=trans)
    ref = A @ (B.t() if trans else B)
    close(C, ref, 2e-5 * np.sqrt(D))
    # MFMA path is exact f32: bitwise deterministic run to run
    C2 = torch.empty_like(C)
    ops.rowgemm(A.float(), B.float(), C2, b_trans=trans)
    assert torch.equal(C, C2)


@pytest.mark.parametrize("D", [64, 256])
def test_rowgemm_asymmetric_identity(D, cuda):
    """A = I (first D rows) with an asymmetric B catches a transposed C-write."""
    M = 3 * D
    A = torch.zeros(M, D, device=cuda)
    A[:D] = torch.eye(D, device=cuda)
    B = torch.arange(D * D, dtype=torch.float32, device=cuda).view(D, D) / (D * D)
    C = torch.empty(M, D, device=cuda)
    ops.rowgemm(A, B, C)
    assert torch.equal(C[:D], B)
    assert torch.equal(C[D:], torch.zeros_like(C[D:]))


@pytest.mark.parametrize("D", DIMS)
def test_rowgemm_combine_epilogue(D, cuda):
    """C = sigmoid(A[a_idx]·S + sum_r W[h,r] * P_r[t]) — the tail-layer forward."""
    g = torch.Generator().manual_seed(11 + D)
    N, M, R = 300, 2049, 3
    X = rnd(N, D, dev=cuda, gen=g, scale=0.2)
    S = rnd(D, D, dev=cuda, gen=g, scale=D ** -0.5)
    W = torch.rand(N, R, generator=g, dtype=torch.float64).to(cuda)
    P = rnd(R, N, D, dev=cuda, gen=g)
    a_idx = torch.randint(0, N, (M,), generator=g).to(cuda)
    h = torch.randint(0, N, (M,), generator=g).to(cuda)
    t = torch.randint(0, N, (M,), generator=g).to(cuda)
    C = torch.empty(M, D, device=cuda)
    ops.rowgemm(X.float(), S.float(), C, a_idx=a_idx.int(), coef=W.float(), coef_idx=h.int(), V=P.float(),
                v_idx=t.int(), v_rel_stride=N * D, act=L.ACT_SIGMOID)
    pre = X[a_idx] @ S
    for r in range(R):
        pre = pre + W[h, r:r + 1] * P[r][t]
    close(C, torch.sigmoid(pre), 2e-5)


@pytest.mark.parametrize("D", DIMS)
def test_rowgemm_rank_update_dsigmoid_accumulate(D, cuda):
    """C = (C + dO·S^T + dz·Wa^T) * X(1-X) — the node-level head backward."""
    g = torch.Generator().manual_seed(13 + D)
    M, R = 777, 4
    dO, S = rnd(M, D, dev=cuda, gen=g), rnd(D, D, dev=cuda, gen=g)
    dz, Wa = rnd(M, R, dev=cuda, gen=g), rnd(D, R, dev=cuda, gen=g)
    X = torch.rand(M, D, generator=g, dtype=torch.float64).to(cuda)
    C0 = rnd(M, D, dev=cuda, gen=g)
    C = C0.float().clone()
    WaT = Wa.t().contiguous().float()
    ops.rowgemm(dO.float(), S.float(), C, b_trans=True, accumulate=True, coef=dz.float(), V=WaT, v_rel_stride=D,
                v_row_stride=0, act=L.ACT_DSIGMOID, aux=X.float())
    ref = (C0 + dO @ S.t() + dz @ Wa.t()) * X * (1 - X)
    close(C, ref, 3e-5 * np.sqrt(D))


@pytest.mark.parametrize("D", DIMS)
def test_gemm_tn(D, cuda):
    g = torch.Generator().manual_seed(17 + D)
    M = 5003
    A, B = rnd(M, D, dev=cuda, gen=g), rnd(M, D, dev=cuda, gen=g)
    C = rnd(D, D, dev=cuda, gen=g).float()
    C0 = C.double().clone()
    slab = torch.empty(ops.tn_blocks(M, D) * D * D, device=cuda)
    ops.gemm_tn(A.float(), B.float(), C, slab, accumulate=True)
    close(C, C0 + A.t() @ B, 2e-6 * np.sqrt(M))
    C1 = torch.empty(D, D, device=cuda)
    ops.gemm_tn(A.float(), B.float(), C1, slab)
    C2 = torch.empty(D, D, device=cuda)
    ops.gemm_tn(A.float(), B.float(), C2, slab)
    assert torch.equal(C1, C2)              # slab reduction in block order: deterministic


@pytest.mark.parametrize("D", [32, 256])
def test_gemm_tn_narrow(D, cuda):
    g = torch.Generator().manual_seed(19 + D)
    M, R = 9001, 3
    A, dz = rnd(M, D, dev=cuda, gen=g), rnd(M, R, dev=cuda, gen=g)
    dWa, dba = torch.empty(D, R, device=cuda), torch.empty(R, device=cuda)
    slab = torch.empty((ops.tn_narrow_blocks(M) + 1) * (D + 1) * R, device=cuda)
    ops.gemm_tn_narrow(A.float(), dz.float(), dWa, dba, slab)
    close(dWa, A.t() @ dz, 2e-6 * np.sqrt(M))
    close(dba, dz.sum(0), 2e-6 * np.sqrt(M))


@pytest.mark.parametrize("D", DIMS)
def test_alpha(D, cuda):
    g = torch.Generator().manual_seed(23 + D)
    M, R = 999, 4
    X, Wa, ba = rnd(M, D, dev=cuda, gen=g), rnd(D, R, dev=cuda, gen=g, scale=0.2), rnd(R, dev=cuda, gen=g)
    S, W = torch.empty(M, R, device=cuda), torch.empty(M, R, device=cuda)
    ops.alpha_fwd(X.float(), Wa.float(), ba.float(), S, W)
    s = torch.softmax(X @ Wa + ba, -1)
    close(S, s, 1e-5)
    close(W, torch.sigmoid(s), 1e-5)
    idx = torch.randint(0, M, (50,), generator=g).to(cuda)
    S2, W2 = torch.empty(50, R, device=cuda), torch.empty(50, R, device=cuda)
    ops.alpha_fwd(X.float(), Wa.float(), ba.float(), S2, W2, x_idx=idx.int())
    assert torch.equal(S2, S[idx]) and torch.equal(W2, W[idx])


@pytest.mark.parametrize("D", DIMS)
def test_combine(D, cuda):
    g = torch.Generator().manual_seed(29 + D)
    N, M, R = 200, 3001, 2
    Y, P = rnd(N, D, dev=cuda, gen=g), rnd(R, N, D, dev=cuda, gen=g)
    W = torch.rand(N, R, generator=g, dtype=torch.float64).to(cuda)
    h = torch.randint(0, N, (M,), generator=g).to(cuda)
    t = torch.randint(0, N, (M,), generator=g).to(cuda)
    out = torch.empty(M, D, device=cuda)
    ops.combine(Y.float(), W.float(), P.float(), out, y_idx=t.int(), coef_idx=h.int(), v_idx=t.int())
    ref = Y[t] + sum(W[h, r:r + 1] * P[r][t] for r in range(R))
    close(out, torch.sigmoid(ref), 1e-5)


@pytest.mark.parametrize("R", [0, 1, 2, 3, 4])
@pytest.mark.parametrize("M,order", [(1, "sorted"), (63, "sorted"), (65, "unsorted"), (20_011, "sorted"),
                                     (20_011, "unsorted"), (20_011, "one_run")])
def test_combine_runs(R, M, order, cuda):
    """Run-combine path (D = 256, y_idx is v_idx, per-edge coef): equal to torch and bitwise to the
    generic edge-parallel kernel (reached by passing a copy of the index as v_idx)."""
    g = torch.Generator().manual_seed(1000 * R + M)
    N, D = 300, 256
    Y, P = rnd(N, D, dev=cuda, gen=g).float(), rnd(max(R, 1), N, D, dev=cuda, gen=g).float()[:R]
    W = torch.rand(M, R, generator=g).to(cuda)
    t = torch.randint(0, N, (M,), generator=g)
    if order == "sorted":
        t = t.sort().values
    elif order == "one_run":
        t = torch.full((M,), 7)
    t = t.to(cuda).int()
    out = torch.empty(M, D, device=cuda)
    ops.combine(Y, W, P, out, y_idx=t, v_idx=t, v_rel_stride=N * D)
    ref = Y.double()[t.long()]
    for r in range(R):
        ref = ref + W.double()[:, r:r + 1] * P.double()[r][t.long()]
    close(out, torch.sigmoid(ref), 1e-5)
    out2 = torch.empty_like(out)
    ops.combine(Y, W, P, out2, y_idx=t, v_idx=t.clone(), v_rel_stride=N * D)
    assert torch.equal(out, out2)


@pytest.mark.parametrize("D", DIMS)
def test_distmult_bce_matches_autograd(D, cuda):
    g = torch.Generator().manual_seed(31 + D)
    N, T, R = 400, 5000, 3
    Xh = torch.rand(N, D, generator=g, dtype=torch.float64).to(cuda)
    Xt = torch.rand(T, D, generator=g, dtype=torch.float64).to(cuda)
    rel = rnd(R, D, dev=cuda, gen=g, scale=0.3)
    h = torch.randint(0, N, (T,), generator=g).to(cuda)
    r = torch.randint(0, R, (T,), generator=g).to(cuda)
    y = (torch.rand(T, generator=g) < 0.5).double().to(cuda)
    scale = 1.0 / (T * N)
    nb = ops.distmult_blocks(T)
    p, ds, do = torch.empty(T, device=cuda), torch.empty(T, device=cuda), torch.empty(T, D, device=cuda)
    drel_slab, loss_slab = torch.empty(nb * R * D, device=cuda), torch.empty(nb, device=cuda)
    ops.distmult_bce(Xh.float(), h.int(), Xt.float(), r.int(), rel.float(), y=y.float(), scale=scale, p_out=p,
                     ds_out=ds, do_out=do, drel_slab=drel_slab, loss_slab=loss_slab)
    drel, loss = torch.empty(R, D, device=cuda), torch.empty(1, device=cuda)
    ops.reduce_slabs(drel_slab, nb, drel)
    ops.reduce_slabs(loss_slab, nb, loss)
    # torch reference: Keras BCE with eps clip, x 1/N, gradient w.r.t. rel and the tail pre-activation
    xt = Xt.clone().requires_grad_(True)
    relv = rel.clone().requires_grad_(True)
    s = (Xh[h] * relv[r] * xt).sum(-1)
    pr = torch.sigmoid(s)
    eps = 1e-7
    pc = pr.clamp(eps, 1 - eps)
    bce = -(y * torch.log(pc + eps) + (1 - y) * torch.log(1 - pc + eps))
    (bce.mean() / N).backward()
    close(p, pr.detach(), 1e-6)
    assert abs(loss.item() / T - bce.mean().item()) < 1e-5
    close(drel, relv.grad, 1e-4)
    close(do, xt.grad * Xt * (1 - Xt), 1e-4)
    # predict-only mode writes p and nothing else
    p2 = torch.empty(T, device=cuda)
    ops.distmult_bce(Xh.float(), h.int(), Xt.float(), r.int(), rel.float(), p_out=p2)
    assert torch.equal(p, p2)


@pytest.mark.parametrize("D", DIMS)
@pytest.mark.parametrize("R,skew", [(1, False), (3, True), (5, False)])
def test_distmult_bce_heads_fused(D, R, skew, cuda):
    """One-pass head-grouped form == distmult_bce + seg_gather_reduce: p / ds / do bitwise, dXh
    bitwise at D=256 (one edge slot per head) and to 1e-5 of max|dXh| below (the head's edges are split over
    64/(D/4) slots), drel / loss to rounding (partial sums visit edges in head order)."""
    g = torch.Generator().manual_seed(41 + D + R)
    N, T = 300, 7001
    Xh = torch.rand(N, D, generator=g).to(cuda)
    Xt = torch.rand(T, D, generator=g).to(cuda)
    rel = (torch.randn(R, D, generator=g) * 0.3).to(cuda)
    if skew:   # a few very hot heads, many heads without edges
        h = torch.where(torch.rand(T, generator=g) < 0.5, torch.randint(0, 3, (T,), generator=g),
                        torch.randint(0, N // 2, (T,), generator=g))
    else:
        h = torch.randint(0, N, (T,), generator=g)
    r = torch.randint(0, R, (T,), generator=g)
    y = (torch.rand(T, generator=g) < 0.5).float().to(cuda)
    hperm = torch.argsort(h, stable=True)
    hptr = torch.searchsorted(h[hperm], torch.arange(N + 1), right=False).to(torch.int32).to(cuda)
    h, r, hperm = h.int().to(cuda), r.int().to(cuda), hperm.int().to(cuda)
    scale = 1.0 / (T * N)
    nb = ops.distmult_blocks(T)
    p, ds, do = torch.empty(T, device=cuda), torch.empty(T, device=cuda), torch.empty(T, D, device=cuda)
    sl_r, sl_l = torch.empty(nb * R * D, device=cuda), torch.empty(nb, device=cuda)
    ops.distmult_bce(Xh, h, Xt, r, rel, y=y, scale=scale, p_out=p, ds_out=ds, do_out=do, drel_slab=sl_r,
                     loss_slab=sl_l)
    dXh = torch.empty(N, D, device=cuda)
    ops.seg_gather_reduce(hptr, Xt, dXh, perm=hperm, coef=ds, r_idx=r, rel=rel, X=Xh)
    drel, loss = torch.empty(R, D, device=cuda), torch.empty(1, device=cuda)
    ops.reduce_slabs(sl_r, nb, drel)
    ops.reduce_slabs(sl_l, nb, loss)

    p2, ds2 = torch.full((T,), 7.0, device=cuda), torch.full((T,), 7.0, device=cuda)
    do2, dXh2 = torch.full((T, D), 7.0, device=cuda), torch.full((N, D), 7.0, device=cuda)
    sl_r2, sl_l2 = torch.empty(nb * R * D, device=cuda), torch.empty(nb, device=cuda)
    ops.distmult_bce_heads(hptr, hperm, Xh, Xt, r, rel, y, do2, dXh2, sl_r2, sl_l2, scale=scale, p_out=p2,
                           ds_out=ds2)
    drel2, loss2 = torch.empty(R, D, device=cuda), torch.empty(1, device=cuda)
    ops.reduce_slabs(sl_r2, nb, drel2)
    ops.reduce_slabs(sl_l2, nb, loss2)
    assert torch.equal(p, p2) and torch.equal(ds, ds2)
    assert torch.equal(do, do2)
    if D == 256:                            # one edge slot per head: the same sequential sum
        assert torch.equal(dXh, dXh2)       # includes zero rows of heads without edges
    else:                                   # 64/(D/4) edge slots per head, partials summed at the end
        assert (dXh2.double() - dXh.double()).abs().max() <= 1e-5 * dXh.double().abs().max()
        empty = (hptr[1:] == hptr[:-1]).nonzero().flatten()
        assert torch.equal(dXh2[empty], torch.zeros_like(dXh2[empty]))
    close(drel2, drel.double(), 1e-5)
    assert abs(loss2.item() - loss.item()) <= 1e-5 * abs(loss.item())


@pytest.mark.parametrize("D", DIMS)
def test_segment_reductions(D, cuda):
    """seg_gather_reduce / tail_seg_reduce / head_bwd_node against index_add references."""
    g = torch.Generator().manual_seed(37 + D)
    N, T, R = 257, 6000, 3
    t = torch.sort(torch.randint(0, N, (T,), generator=g)).values
    h = torch.randint(0, N, (T,), generator=g)
    tptr = torch.searchsorted(t, torch.arange(N + 1), right=False).to(torch.int32).to(cuda)
    hperm = torch.argsort(h, stable=True)
    hptr = torch.searchsorted(h[hperm], torch.arange(N + 1), right=False).to(torch.int32).to(cuda)
    t, h, hperm = t.to(cuda), h.to(cuda), hperm.to(cuda)
    rows = rnd(T, D, dev=cuda, gen=g)
    coef = rnd(T, dev=cuda, gen=g)
    r_idx = torch.randint(0, R, (T,), generator=g).to(cuda)
    rel = rnd(R, D, dev=cuda, gen=g)
    X = torch.rand(N, D, generator=g, dtype=torch.float64).to(cuda)
    out = torch.empty(N, D, device=cuda)
    ops.seg_gather_reduce(hptr, rows.float(), out, perm=hperm.int(), coef=coef.float(), r_idx=r_idx.int(),
                          rel=rel.float(), X=X.float())
    ref = torch.zeros(N, D, dtype=torch.float64, device=cuda).index_add_(0, h, coef[:, None] * rel[r_idx] * rows)
    close(out, ref * X * (1 - X), 1e-5)

    W = torch.rand(N, R, generator=g, dtype=torch.float64).to(cuda)
    P = rnd(R, N, D, dev=cuda, gen=g)
    dO = rnd(T, D, dev=cuda, gen=g)
    dP, dWe, dsum = torch.empty(R, N, D, device=cuda), torch.empty(T, R, device=cuda), torch.empty(N, D, device=cuda)
    ops.tail_seg_reduce(tptr, h.int(), W.float(), dO.float(), P.float(), dP, dWe, dsum=dsum)
    for r in range(R):
        close(dP[r], torch.zeros(N, D, dtype=torch.float64, device=cuda).index_add_(0, t, W[h, r:r + 1] * dO), 1e-5)
        close(dWe[:, r], (dO * P[r][t]).sum(-1), 1e-5)
    close(dsum, torch.zeros(N, D, dtype=torch.float64, device=cuda).index_add_(0, t, dO), 1e-5)

    dOn = rnd(N, D, dev=cuda, gen=g)
    Ssm = torch.softmax(rnd(N, R, dev=cuda, gen=g), -1)
    Wn = torch.sigmoid(Ssm)
    dP0 = dP.clone()
    dsum0 = dsum.clone()
    dz = torch.empty(N, R, device=cuda)
    ops.head_bwd_node(dOn.float(), P.float(), Ssm.float(), Wn.float(), dP, dz, hseg_ptr=hptr, hperm=hperm.int(),
                      dWedge=dWe, dsum=dsum)
    dWn = (dOn[None] * P).sum(-1).t() + torch.zeros(N, R, dtype=torch.float64, device=cuda).index_add_(0, h, dWe.double())
    s_ = Ssm.clone().requires_grad_(True)
    (torch.sigmoid(s_) * dWn).sum().backward()
    ds = s_.grad
    dz_ref = Ssm * (ds - (ds * Ssm).sum(-1, keepdim=True))
    close(dz, dz_ref, 1e-5)
    close(dP, dP0.double() + Wn.t()[:, :, None] * dOn[None], 1e-5)
    close(dsum, dsum0.double() + dOn, 1e-6)


def test_adam_kernel_matches_keras_forms(cuda):
    g = torch.Generator().manual_seed(41)
    n = 10001
    var, gr = torch.randn(n, generator=g).to(cuda), torch.randn(n, generator=g).to(cuda) * 1e-3
    m, v = torch.randn(n, generator=g).abs().to(cuda) * 1e-3, torch.rand(n, generator=g).to(cuda) * 1e-6
    b1, b2, eps, alpha = 0.9, 0.999, 1e-7, 3e-4
    for sparse in (0, 1):
        var2, m2, v2 = var.clone(), m.clone(), v.clone()
        ops.adam(var2, m2, v2, gr, alpha, b1, b2, eps, sparse)
        vd, md, vvd, gd = var.double(), m.double(), v.double(), gr.double()
        mr = md * b1 + gd * (1 - b1)
        vr = vvd * b2 + gd * gd * (1 - b2)
        close(m2, mr, 1e-6)
        close(v2, vr, 1e-6)
        close(var2, vd - alpha * mr / (vr.sqrt() + eps), 1e-6)


def _run_structured_idx(M, N, gen):
    """Row indices whose 32-row tiles hold 1, 2, 8, 15, 16, 17, 24 and 32 runs of equal values
    (the D=256 row GEMM keeps at most 16 distinct V rows of a tile in LDS for its second relation
    and reads the rest of such a tile from global memory)."""
    idx = torch.empty(M, dtype=torch.int64)
    run = 0
    for t0 in range(0, M, 32):
        rows = min(32, M - t0)
        u = min([1, 2, 8, 15, 16, 17, 24, 32][(t0 // 32) % 8], rows)
        cuts = sorted(torch.randperm(rows - 1, generator=gen)[:u - 1].add(1).tolist())
        for k, (a, b) in enumerate(zip([0] + cuts, cuts + [rows])):
            idx[t0 + a:t0 + b] = (run + k) % N
        run += u
    return idx


@pytest.mark.parametrize("mode", ["zero_coef", "combine", "combine_r1", "combine_runs", "accumulate", "gatherA",
                                  "small_M"])
def test_rowgemm_v3_exact_bitwise_equals_register_kernel(mode, cuda):
    """D=256 exact mode: the pipelined v3 kernel == the register-staged kernel, bit for bit (the same k-ordered
    MFMA fmaf chain, the same epilogue order), including a ragged last tile and multi-tile persistent blocks.
    The register-staged kernel is reached by storing the V rows with a padded row stride (the v3 kernel takes
    dense rows only); "zero_coef" (coefficients 0: the plain GEMM) compares the MFMA chains alone."""
    g = torch.Generator().manual_seed(43)
    D, N, M, R = 256, 700, (77 if mode == "small_M" else 40_000 + 17), (1 if mode == "combine_r1" else 2)
    A = torch.randn(M, D, generator=g).to(cuda)
    S = (torch.randn(D, D, generator=g) / 16).to(cuda)
    coef = torch.rand(N, R, generator=g).to(cuda)
    if mode == "zero_coef":
        coef.zero_()
    v_idx = _run_structured_idx(M, N, g) if mode == "combine_runs" else torch.randint(0, N, (M,), generator=g)
    kw = dict(coef=coef, coef_idx=torch.randint(0, N, (M,), generator=g).int().to(cuda), v_idx=v_idx.int().to(cuda),
              act=L.ACT_SIGMOID)
    if mode == "accumulate":
        kw.update(accumulate=True, b_trans=True, act=L.ACT_NONE)
    elif mode == "gatherA":
        kw.update(a_idx=torch.randint(0, M, (M,), generator=g).int().to(cuda))
    V = torch.randn(R, N, D, generator=g).to(cuda)
    Vpad = torch.zeros(R, N, 2 * D, device=cuda)
    Vpad[:, :, :D] = V
    C0 = torch.randn(M, D, generator=g).to(cuda)
    out = []
    for Vt, vrs, kid in ((V, D, 300 + 10 * R + 2), (Vpad, 2 * D, 100)):
        kv = dict(kw, V=Vt, v_row_stride=vrs, v_rel_stride=N * vrs)
        assert ops.rowgemm_kernel_id(A, S, C0, **kv) == kid
        C = C0.clone()
        ops.rowgemm(A, S, C, **kv)
        out.append(C)
    assert torch.equal(out[0], out[1])


def _maxrel(got, ref):
    return ((got.double() - ref).abs().max() / ref.abs().max()).item()


@pytest.mark.parametrize("D", DIMS)
def test_rowgemm_batched_equals_single_calls(D, cuda):
    """iddgcn_rowgemm_batched_f32 (one launch for D < 256) == the same GEMMs one call at a time,
    bitwise: different row counts (one empty), plain / transposed-accumulate / combine epilogues."""
    g = torch.Generator().manual_seed(3 * D)
    N, R = 120, 2
    calls = []
    for k, M in enumerate([845, 77, 0, 4000, 845]):
        A = torch.randn(max(M, 1), D, generator=g).to(cuda)
        B = (torch.randn(D, D, generator=g) / D ** 0.5).to(cuda)
        kw = {}
        if k == 1:
            kw = dict(b_trans=True, accumulate=True)
        elif k == 3:
            kw = dict(coef=torch.rand(N, R, generator=g).to(cuda), coef_idx=torch.randint(0, N, (M,), generator=g).int().to(cuda),
                      V=torch.randn(R, N, D, generator=g).to(cuda), v_idx=torch.randint(0, N, (M,), generator=g).int().to(cuda),
                      v_rel_stride=N * D, act=L.ACT_SIGMOID)
        C0 = torch.randn(M, D, generator=g).to(cuda)
        calls.append((A, B, C0, kw))
    single, batched = [], []
    for A, B, C0, kw in calls:
        C = C0.clone()
        ops.rowgemm(A, B, C, M=C.shape[0], **kw)
        single.append(C)
    outs = [C0.clone() for _, _, C0, _ in calls]
    ops.rowgemm_batched([(A, B, C, dict(kw, M=C.shape[0])) for (A, B, _, kw), C in zip(calls, outs)])
    for a, b in zip(single, outs):
        assert torch.equal(a, b)


@pytest.mark.parametrize("mode", ["plain", "trans", "combine", "combine_r1", "combine_runs", "dsig", "rank_bcast",
                                  "accumulate", "gatherA", "small_M", "row_decades", "zero_rows"])
def test_rowgemm_split_f16_vs_fp64(mode, cuda):
    """Split-fp16 operand mode (D=256): error vs an fp64 torch reference no larger than twice the
    exact-f32 MFMA path's (floor 1e-6 of max|ref|), on every epilogue form, ragged tiles, rows whose
    magnitudes span 12 decades (per-row scales) and all-zero rows; deterministic run to run."""
    g = torch.Generator().manual_seed(sum(map(ord, mode)))
    D, N, R = 256, 700, (1 if mode == "combine_r1" else 2)
    M = 77 if mode == "small_M" else 20_000 + 17
    A = torch.rand(M, D, generator=g, dtype=torch.float64)
    if mode == "row_decades":
        A = torch.randn(M, D, generator=g, dtype=torch.float64) * 10 ** (12 * torch.rand(M, 1, generator=g,
                                                                                        dtype=torch.float64) - 6)
    if mode == "zero_rows":
        A[::3] = 0
    S = torch.randn(D, D, generator=g, dtype=torch.float64)
    A, S = A.to(cuda), S.to(cuda)
    kw, C0 = {}, None
    Af, Sf = A.float(), S.float()
    if mode in ("combine", "combine_r1", "combine_runs"):
        W = torch.rand(N, R, generator=g, dtype=torch.float64).to(cuda)
        P = (torch.randn(R, N, D, generator=g, dtype=torch.float64) * 4).to(cuda)
        h = torch.randint(0, N, (M,), generator=g).to(cuda)
        t = torch.randint(0, N, (M,), generator=g).sort().values.to(cuda)
        if mode == "combine_runs":
            t = _run_structured_idx(M, N, g).to(cuda)
        kw = dict(coef=W.float(), coef_idx=h.int(), V=P.float(), v_idx=t.int(), v_rel_stride=N * D,
                  act=L.ACT_SIGMOID)
        ref = torch.sigmoid(A @ S + sum(W[h, r:r + 1] * P[r][t] for r in range(R)))
    elif mode == "dsig":
        X = torch.rand(M, D, generator=g, dtype=torch.float64).to(cuda)
        kw = dict(b_trans=True, act=L.ACT_DSIGMOID, aux=X.float())
        ref = (A @ S.t()) * X * (1 - X)
    elif mode in ("rank_bcast", "bcast", "bcast_r1"):
        # dO S^T + dz W_a^T (broadcast V: one row per relation for every output row), with the sigma' factor
        # (head-chain backward, layers 2-3) or without (dE, layer 1)
        Rb = 1 if mode == "bcast_r1" else R
        X = torch.rand(M, D, generator=g, dtype=torch.float64).to(cuda)
        dz = torch.randn(M, Rb, generator=g, dtype=torch.float64).to(cuda)
        Wa = torch.randn(D, Rb, generator=g, dtype=torch.float64).to(cuda)
        kw = dict(b_trans=True, coef=dz.float(), V=Wa.t().contiguous().float(), v_rel_stride=D, v_row_stride=0)
        ref = A @ S.t() + dz @ Wa.t()
        kid = 502
        if mode == "rank_bcast":
            kw.update(act=L.ACT_DSIGMOID, aux=X.float())
            ref = ref * X * (1 - X)
            kid = 503
    elif mode in ("accumulate", "accumulate_trans", "accumulate_sigmoid"):
        C0 = torch.randn(M, D, generator=g, dtype=torch.float64).to(cuda)
        kw = dict(accumulate=True, b_trans=mode == "accumulate_trans")
        ref = C0 + A @ (S.t() if mode == "accumulate_trans" else S)
        if mode == "accumulate_sigmoid":
            kw.update(act=L.ACT_SIGMOID)
            ref = torch.sigmoid(ref)
        kid = 501
    elif mode == "gatherA":
        ai = torch.randint(0, M, (M,), generator=g).to(cuda)
        kw = dict(a_idx=ai.int())
        ref = A[ai] @ S
    elif mode == "trans":
        kw = dict(b_trans=True)
        ref = A @ S.t()
    else:
        ref = A @ S
    errs, outs = {}, {}
    for gm in (L.GEMM_EXACT_F32, L.GEMM_SPLIT_F16):
        C = C0.float().clone() if C0 is not None else torch.full((M, D), 7.0, device=cuda)
        ops.rowgemm(Af, Sf, C, precision=gm, **kw)
        if gm == L.GEMM_SPLIT_F16:
            C2 = C0.float().clone() if C0 is not None else torch.empty(M, D, device=cuda)
            ops.rowgemm(Af, Sf, C2, precision=gm, **kw)
            assert torch.equal(C, C2)
        outs[gm], errs[gm] = C, _maxrel(C, ref)
    split = outs[L.GEMM_SPLIT_F16]
    if mode == "zero_rows":
        assert torch.equal(split[::3], torch.zeros_like(split[::3]))
    if mode == "row_decades":   # per-row relative error, every row (per-row scales)
        rel = ((split.double() - ref).abs().amax(1) / ref.abs().amax(1)).max().item()
        assert rel <= 1e-5, rel
    assert errs[L.GEMM_SPLIT_F16] <= max(2 * errs[L.GEMM_EXACT_F32], 1e-6), errs


@pytest.mark.parametrize("M,kind", [(31, "plain"), (5003, "plain"), (300_017, "decades"), (70_001, "zero_blocks"),
                                    (40_000, "growing")])
def test_gemm_tn_split_f16_vs_fp64(M, kind, cuda):
    """Split-fp16 TN GEMM (running per-block power-of-two scales): error vs fp64 within 2x the exact
    path's (floor 1e-6), with row magnitudes spanning decades, all-zero stretches, and magnitudes that
    change along the rows (block scales lowered many times); deterministic run to run."""
    g = torch.Generator().manual_seed(M)
    D = 256
    A = torch.rand(M, D, generator=g, dtype=torch.float64)
    B = torch.randn(M, D, generator=g, dtype=torch.float64) * 1e-12
    if kind == "decades":
        B = B * 10 ** (6 * torch.rand(M, 1, generator=g, dtype=torch.float64) - 3)
    elif kind == "zero_blocks":
        B[: M // 2] = 0
        A[M // 3: M // 2] = 0
    elif kind == "growing":
        B = B * torch.logspace(-4, 4, M, dtype=torch.float64)[:, None]
        A = A * torch.logspace(3, -3, M, dtype=torch.float64)[:, None]
    A, B = A.to(cuda), B.to(cuda)
    ref = A.t() @ B
    slab = torch.empty(ops.tn_blocks(M, D) * D * D, device=cuda)
    errs = {}
    for gm in (L.GEMM_EXACT_F32, L.GEMM_SPLIT_F16):
        C = torch.empty(D, D, device=cuda)
        ops.gemm_tn(A.float(), B.float(), C, slab, precision=gm)
        errs[gm] = _maxrel(C, ref)
        if gm == L.GEMM_SPLIT_F16:
            C2 = torch.empty(D, D, device=cuda)
            ops.gemm_tn(A.float(), B.float(), C2, slab, precision=gm)
            assert torch.equal(C, C2)
    assert errs[L.GEMM_SPLIT_F16] <= max(2 * errs[L.GEMM_EXACT_F32], 1e-6), errs


B3_FORMS = ["plain", "trans", "combine", "combine_r1", "combine_runs", "combine_random", "dsig", "small_M",
            "tiny_M", "row_decades", "zero_rows", "accumulate", "accumulate_trans", "rank_bcast", "bcast",
            "bcast_r1"]
B3_FALLBACK = ["gatherA", "coef_idx", "accumulate_sigmoid"]


@pytest.mark.parametrize("mode", B3_FORMS + B3_FALLBACK)
def test_rowgemm_bf16x3_vs_fp64(mode, cuda):
    """bf16x3 operand mode (IDDGCN_GEMM_BF16X3, D = 256: every fp32 operand split exactly into three bf16
    pieces, six bf16 MFMA products, fp32 accumulation): error vs an fp64 torch reference within 1.25x the
    exact-f32 MFMA path's (floor 1e-6 of max|ref|) on every form the bf16x3 kernel takes (the column-half
    kernel is asserted: 500 + 10 NV + aux), incl. ragged and tiny M, tiles with up to 32 distinct gathered rows,
    rows spanning 12 decades (per-row error 1e-5), zero rows, C += A B (in place, the old C rows through the
    aux slab) and broadcast V rows (dz W_a^T, R = 1, 2, with and without the sigma' factor); deterministic run
    to run.  The forms it does not take (gathered A, coef_idx, accumulate with an activation) run the exact
    kernel: bitwise the exact mode."""
    g = torch.Generator().manual_seed(sum(map(ord, mode)) + 7)
    D, N, R = 256, 700, (1 if mode == "combine_r1" else 2)
    M = {"small_M": 77, "tiny_M": 5}.get(mode, 20_000 + 17)
    A = torch.rand(M, D, generator=g, dtype=torch.float64)
    if mode == "row_decades":
        A = torch.randn(M, D, generator=g, dtype=torch.float64) * 10 ** (12 * torch.rand(M, 1, generator=g,
                                                                                        dtype=torch.float64) - 6)
    if mode == "zero_rows":
        A[::3] = 0
    S = torch.randn(D, D, generator=g, dtype=torch.float64)
    A, S = A.to(cuda), S.to(cuda)
    kw, C0 = {}, None
    Af, Sf = A.float(), S.float()
    kid = 500
    if mode in ("combine", "combine_r1", "combine_runs", "combine_random", "coef_idx"):
        W = torch.rand(N, R, generator=g, dtype=torch.float64).to(cuda)
        P = (torch.randn(R, N, D, generator=g, dtype=torch.float64) * 4).to(cuda)
        h = torch.randint(0, N, (M,), generator=g).to(cuda)
        t = torch.randint(0, N, (M,), generator=g).sort().values.to(cuda)
        if mode == "combine_runs":
            t = _run_structured_idx(M, N, g).to(cuda)
        if mode == "combine_random":        # up to 32 distinct gathered rows per tile (two DMA rounds)
            t = torch.randint(0, N, (M,), generator=g).to(cuda)
        if mode == "coef_idx":
            kw = dict(coef=W.float(), coef_idx=h.int())
        else:
            kw = dict(coef=W[h].float().contiguous())
        kw.update(V=P.float(), v_idx=t.int(), v_rel_stride=N * D, act=L.ACT_SIGMOID)
        ref = torch.sigmoid(A @ S + sum(W[h, r:r + 1] * P[r][t] for r in range(R)))
        kid = 500 + 10 * R
    elif mode == "dsig":
        X = torch.rand(M, D, generator=g, dtype=torch.float64).to(cuda)
        kw = dict(b_trans=True, act=L.ACT_DSIGMOID, aux=X.float())
        ref = (A @ S.t()) * X * (1 - X)
        kid = 501
    elif mode in ("rank_bcast", "bcast", "bcast_r1"):
        # dO S^T + dz W_a^T (broadcast V: one row per relation for every output row), with the sigma' factor
        # (head-chain backward, layers 2-3) or without (dE, layer 1)
        Rb = 1 if mode == "bcast_r1" else R
        X = torch.rand(M, D, generator=g, dtype=torch.float64).to(cuda)
        dz = torch.randn(M, Rb, generator=g, dtype=torch.float64).to(cuda)
        Wa = torch.randn(D, Rb, generator=g, dtype=torch.float64).to(cuda)
        kw = dict(b_trans=True, coef=dz.float(), V=Wa.t().contiguous().float(), v_rel_stride=D, v_row_stride=0)
        ref = A @ S.t() + dz @ Wa.t()
        kid = 502
        if mode == "rank_bcast":
            kw.update(act=L.ACT_DSIGMOID, aux=X.float())
            ref = ref * X * (1 - X)
            kid = 503
    elif mode in ("accumulate", "accumulate_trans", "accumulate_sigmoid"):
        C0 = torch.randn(M, D, generator=g, dtype=torch.float64).to(cuda)
        kw = dict(accumulate=True, b_trans=mode == "accumulate_trans")
        ref = C0 + A @ (S.t() if mode == "accumulate_trans" else S)
        if mode == "accumulate_sigmoid":
            kw.update(act=L.ACT_SIGMOID)
            ref = torch.sigmoid(ref)
        kid = 501
    elif mode == "gatherA":
        ai = torch.randint(0, M, (M,), generator=g).to(cuda)
        kw = dict(a_idx=ai.int())
        ref = A[ai] @ S
    elif mode == "trans":
        kw = dict(b_trans=True)
        ref = A @ S.t()
    else:
        ref = A @ S
    errs, outs = {}, {}
    for gm in (L.GEMM_EXACT_F32, L.GEMM_BF16X3):
        C = C0.float().clone() if C0 is not None else torch.full((M, D), 7.0, device=cuda)
        ops.rowgemm(Af, Sf, C, precision=gm, **kw)
        if gm == L.GEMM_BF16X3:
            C2 = C0.float().clone() if C0 is not None else torch.empty(M, D, device=cuda)
            ops.rowgemm(Af, Sf, C2, precision=gm, **kw)
            assert torch.equal(C, C2)
        outs[gm], errs[gm] = C, _maxrel(C, ref)
    b3 = outs[L.GEMM_BF16X3]
    if mode in B3_FALLBACK:
        assert ops.rowgemm_kernel_id(Af, Sf, b3, precision="bf16x3", **kw) < 500
        assert torch.equal(b3, outs[L.GEMM_EXACT_F32])
        return
    assert ops.rowgemm_kernel_id(Af, Sf, b3, precision="bf16x3", **kw) == kid
    if mode == "zero_rows":
        assert torch.equal(b3[::3], torch.zeros_like(b3[::3]))
    if mode == "row_decades":
        rel = ((b3.double() - ref).abs().amax(1) / ref.abs().amax(1)).max().item()
        assert rel <= 1e-5, rel
    assert errs[L.GEMM_BF16X3] <= max(1.25 * errs[L.GEMM_EXACT_F32], 1e-6), errs


@pytest.mark.parametrize("M,kind", [(31, "plain"), (5003, "plain"), (300_017, "decades"), (70_001, "zero_blocks"),
                                    (40_000, "growing"), (16, "plain"), (1, "plain")])
def test_gemm_tn_bf16x3_vs_fp64(M, kind, cuda):
    """bf16x3 TN GEMM (16-row tiles, transposed LDS reads of the three planes): error vs fp64 within 1.25x the
    exact path's (floor 1e-6), rows spanning decades, zero stretches, growing magnitudes, ragged and one-row
    M; deterministic run to run."""
    g = torch.Generator().manual_seed(M + 3)
    D = 256
    A = torch.rand(M, D, generator=g, dtype=torch.float64)
    B = torch.randn(M, D, generator=g, dtype=torch.float64) * 1e-12
    if kind == "decades":
        B = B * 10 ** (6 * torch.rand(M, 1, generator=g, dtype=torch.float64) - 3)
    elif kind == "zero_blocks":
        B[: M // 2] = 0
        A[M // 3: M // 2] = 0
    elif kind == "growing":
        B = B * torch.logspace(-4, 4, M, dtype=torch.float64)[:, None]
        A = A * torch.logspace(3, -3, M, dtype=torch.float64)[:, None]
    A, B = A.to(cuda), B.to(cuda)
    ref = A.t() @ B
    slab = torch.empty(ops.tn_blocks(M, D) * D * D, device=cuda)
    errs = {}
    for gm in (L.GEMM_EXACT_F32, L.GEMM_BF16X3):
        C = torch.empty(D, D, device=cuda)
        ops.gemm_tn(A.float(), B.float(), C, slab, precision=gm)
        errs[gm] = _maxrel(C, ref)
        if gm == L.GEMM_BF16X3:
            C2 = torch.empty(D, D, device=cuda)
            ops.gemm_tn(A.float(), B.float(), C2, slab, precision=gm)
            assert torch.equal(C, C2)
    assert errs[L.GEMM_BF16X3] <= max(1.25 * errs[L.GEMM_EXACT_F32], 1e-6), errs


def _tail_runs(lengths, M):
    """Sorted row indices built from consecutive runs of the given lengths (tail-sorted edges)."""
    idx = torch.repeat_interleave(torch.arange(len(lengths)), torch.as_tensor(lengths))[:M]
    return idx


@pytest.mark.parametrize("R", [3, 4, 5, 8])
@pytest.mark.parametrize("gm", ["exact", "split"])
@pytest.mark.parametrize("order", ["tail_runs", "structured", "identity", "random"])
def test_rowgemm256_many_relations_gather(R, gm, order, cuda):
    """The D=256 row GEMM with a gathered combine of R > 2 relations (BASELINE config 5: R = 8): capped
    gather slabs (7 distinct V rows per relation per 32-row tile in LDS, further ones read from L2),
    run-time R below the slot capacity (R = 3, 5).  Row orders: tail-sorted runs (the edge forward),
    tiles with 1..32 runs, identity rows (the node-level head chain: 32 distinct rows per tile) and
    random rows.  vs fp64: exact path 2e-5, split path <= 2x the exact path's error."""
    g = torch.Generator().manual_seed(100 + R + len(order))
    D, N, M = 256, 4000, 30_000 + 5
    if order == "tail_runs":
        t = _tail_runs(torch.randint(6, 60, (N,), generator=g), M)
    elif order == "structured":
        t = _run_structured_idx(M, N, g)
    elif order == "identity":
        N = M
        t = None
    else:
        t = torch.randint(0, N, (M,), generator=g)
    A = torch.rand(M, D, generator=g, dtype=torch.float64).to(cuda)
    S = (torch.randn(D, D, generator=g, dtype=torch.float64) / 16).to(cuda)
    W = torch.rand(M, R, generator=g, dtype=torch.float64).to(cuda)
    P = torch.randn(R, N, D, generator=g, dtype=torch.float64).to(cuda)
    rows = torch.arange(M, device=cuda) if t is None else t.to(cuda)
    ref = torch.sigmoid(A @ S + sum(W[:, r:r + 1] * P[r][rows] for r in range(R)))
    kw = dict(coef=W.float(), V=P.float(), v_idx=None if t is None else rows.int(), v_rel_stride=N * D,
              act=L.ACT_SIGMOID)
    errs = {}
    for mode in (L.GEMM_EXACT_F32, L.GEMM_SPLIT_F16) if gm == "split" else (L.GEMM_EXACT_F32,):
        C = torch.empty(M, D, device=cuda)
        assert ops.rowgemm_kernel_id(A.float(), S.float(), C, precision=mode, **kw) == \
            300 + 10 * (4 if R <= 4 else 8) + 2 + (2000 if mode == L.GEMM_SPLIT_F16 else 0)
        ops.rowgemm(A.float(), S.float(), C, precision=mode, **kw)
        errs[mode] = _maxrel(C, ref)
    assert errs[L.GEMM_EXACT_F32] <= 2e-5, errs
    if gm == "split":
        assert errs[L.GEMM_SPLIT_F16] <= max(2 * errs[L.GEMM_EXACT_F32], 1e-6), errs


@pytest.mark.parametrize("gm", ["exact", "split"])
def test_rowgemm256_many_relations_gather_offsets_past_2e32(gm, cuda):
    """The slot-major V slabs of the R = 8 gathered forward address relation r's row as r·v_rel_stride + the
    row offset: with N = 2.5M nodes ((R-1)·N·D = 4.5e9 elements > 2^32) the last relation's rows sit past 32-bit
    element offsets.  Rows gathered from the top of the table (tail runs), vs fp64 (exact 2e-5; split 2x)."""
    g = torch.Generator(device=cuda).manual_seed(31)
    D, R, N, M = 256, 8, 2_500_000, 4096
    assert (R - 1) * N * D > 2 ** 32
    P = torch.randn(R, N, D, device=cuda, generator=g)
    t = (N - 1 - torch.sort(torch.randint(0, 600, (M,), device=cuda, generator=g), descending=True)[0]).int()
    A = torch.rand(M, D, device=cuda, generator=g)
    S = torch.randn(D, D, device=cuda, generator=g) / 16
    W = torch.rand(M, R, device=cuda, generator=g)
    ref = torch.sigmoid(A.double() @ S.double() + sum(W[:, r:r + 1].double() * P[r][t.long()].double()
                                                      for r in range(R)))
    kw = dict(coef=W, V=P, v_idx=t, v_rel_stride=N * D, act=L.ACT_SIGMOID)
    errs = {}
    for mode in (L.GEMM_EXACT_F32, L.GEMM_SPLIT_F16) if gm == "split" else (L.GEMM_EXACT_F32,):
        C = torch.empty(M, D, device=cuda)
        assert ops.rowgemm_kernel_id(A, S, C, precision=mode, **kw) == \
            300 + 10 * 8 + 2 + (2000 if mode == L.GEMM_SPLIT_F16 else 0)
        ops.rowgemm(A, S, C, precision=mode, **kw)
        errs[mode] = _maxrel(C, ref)
    del P
    torch.cuda.empty_cache()
    assert errs[L.GEMM_EXACT_F32] <= 2e-5, errs
    if gm == "split":
        assert errs[L.GEMM_SPLIT_F16] <= max(2 * errs[L.GEMM_EXACT_F32], 1e-6), errs


@pytest.mark.parametrize("R", [4, 8])
@pytest.mark.parametrize("gm", ["exact", "split"])
def test_rowgemm256_rank_update_many_relations(R, gm, cuda):
    """D=256 node-level head backward with R > 2 (broadcast V rows, up to 8 coefficients per row):
    C = (C + dO·S^T + dz·Wa^T) * X(1-X), on the v3 kernel."""
    g = torch.Generator().manual_seed(7 * R)
    D, M = 256, 9001
    dO, S = rnd(M, D, dev=cuda, gen=g), rnd(D, D, dev=cuda, gen=g, scale=1 / 16)
    dz, Wa = rnd(M, R, dev=cuda, gen=g), rnd(D, R, dev=cuda, gen=g)
    X = torch.rand(M, D, generator=g, dtype=torch.float64).to(cuda)
    C0 = rnd(M, D, dev=cuda, gen=g)
    ref = (C0 + dO @ S.t() + dz @ Wa.t()) * X * (1 - X)
    kw = dict(b_trans=True, accumulate=True, coef=dz.float(), V=Wa.t().contiguous().float(), v_rel_stride=D,
              v_row_stride=0, act=L.ACT_DSIGMOID, aux=X.float(), precision=gm)
    C = C0.float().clone()
    assert ops.rowgemm_kernel_id(dO.float(), S.float(), C, **kw) == 300 + 2 + 1 + 8 + (2000 if gm == "split" else 0)
    ops.rowgemm(dO.float(), S.float(), C, **kw)
    assert _maxrel(C, ref) <= 2e-5


@pytest.mark.parametrize("gm", ["exact", "split"])
def test_rowgemm256_batched_one_launch_bitwise(gm, cuda):
    """D=256 batches whose entries share a v3 variant run as ONE launch (blockIdx.y = entry), bitwise
    equal to one call per entry: ragged row counts (1 row, an empty entry, 100k rows), plain
    projections and transposed-accumulate ones."""
    g = torch.Generator().manual_seed(5)
    D = 256
    for kw in (dict(), dict(b_trans=True, accumulate=True)):
        calls = []
        for M in [5000, 1, 0, 100_003, 777, 32, 4096]:
            A = torch.randn(max(M, 1), D, generator=g).to(cuda)
            B = (torch.randn(D, D, generator=g) / 16).to(cuda)
            calls.append((A, B, torch.randn(M, D, generator=g).to(cuda)))
        kw = dict(kw, precision=gm)
        single = []
        for A, B, C0 in calls:
            C = C0.clone()
            ops.rowgemm(A, B, C, M=C.shape[0], **kw)
            single.append(C)
        outs = [C0.clone() for _, _, C0 in calls]
        ops.rowgemm_batched([(A, B, C, dict(kw, M=C.shape[0])) for (A, B, _), C in zip(calls, outs)])
        for a, b in zip(single, outs):
            assert torch.equal(a, b)


@pytest.mark.parametrize("gm", ["exact", "split"])
def test_rowgemm256_batched_full_projection_set(gm, cuda):
    """A full batch of L.ROWGEMM_BATCH = 25 entries laid out like config 5's forward projections (entry l*R + r
    reads A_r, R = 8, three layers, plus one extra entry): one launch, bitwise equal to one call per entry; one
    entry more is refused.  (The engine-level check is tests/test_gpu_config5.py: its layer-3 tables come from
    entries 16-23.)"""
    g = torch.Generator().manual_seed(9)
    D, R, M = 256, 8, 20_011
    A = [torch.randn(M, D, generator=g).to(cuda) for _ in range(R)] + [torch.randn(M, D, generator=g).to(cuda)]
    calls = [(A[r], (torch.randn(D, D, generator=g) / 16).to(cuda)) for _ in range(3) for r in range(R)]
    calls.append((A[R], (torch.randn(D, D, generator=g) / 16).to(cuda)))
    assert len(calls) == L.ROWGEMM_BATCH
    single = []
    for a, b in calls:
        C = torch.empty(M, D, device=cuda)
        ops.rowgemm(a, b, C, precision=gm)
        single.append(C)
    outs = [torch.full((M, D), float("nan"), device=cuda) for _ in calls]
    ops.rowgemm_batched([(a, b, C, dict(precision=gm)) for (a, b), C in zip(calls, outs)])
    for x, y in zip(single, outs):
        assert torch.equal(x, y)
    with pytest.raises(L.IddgcnError):
        ops.rowgemm_batched([(a, b, C, dict(precision=gm)) for (a, b), C in zip(calls + calls[:1], outs + outs[:1])])


@pytest.mark.parametrize("R", [1, 2, 4, 8])
@pytest.mark.parametrize("case", ["uniform", "hub", "sparse", "empty", "tiny"])
@pytest.mark.parametrize("dsum", [False, True])
def test_tail_seg_per_edge_w(R, case, dsum, cuda):
    """tail_seg_reduce at D = 256 with per-edge W (h_idx = NULL, the training step's form) against float64
    index_add references, and against the same call with h_idx = arange (W[h_idx[e]] = W[e]): dP and dsum
    bitwise equal, dWedge within 1e-6.  Cases: runs of tails with and without edges, a hub tail with a
    third of the edges, almost every tail without edges (3 edges on 300 tails), tiny graphs.  R >= 4 runs the
    software-pipelined one-node-per-wave loop (scalar coefficient loads, next edge group in flight)."""
    g = torch.Generator().manual_seed(11 * R + len(case) + dsum)
    D = 256
    N = {"tiny": 5, "empty": 300}.get(case, 1000 + 7)
    T = {"tiny": 37, "empty": 3, "sparse": 60}.get(case, 30_000)
    t = torch.randint(0, N, (T,), generator=g)
    if case == "hub":
        t[: T // 3] = 517
    if case == "uniform":
        t[(t >= 100) & (t < 140)] = 99            # 40 consecutive tails without edges
    t = torch.sort(t).values
    tptr = torch.searchsorted(t, torch.arange(N + 1), right=False).to(torch.int32).to(cuda)
    W = torch.rand(T, R, generator=g, dtype=torch.float64).to(cuda)
    P = rnd(R, N, D, dev=cuda, gen=g)
    dO = rnd(T, D, dev=cuda, gen=g)
    tc = t.to(cuda)
    dP, dWe = torch.full((R, N, D), 7.0, device=cuda), torch.empty(T, R, device=cuda)
    ds = torch.full((N, D), 7.0, device=cuda) if dsum else None
    ops.tail_seg_reduce(tptr, None, W.float(), dO.float(), P.float(), dP, dWe, dsum=ds)
    for r in range(R):
        close(dP[r], torch.zeros(N, D, dtype=torch.float64, device=cuda).index_add_(0, tc, W[:, r:r + 1] * dO), 1e-5)
        if T:
            close(dWe[:, r], (dO * P[r][tc]).sum(-1), 1e-5)
    if dsum:
        close(ds, torch.zeros(N, D, dtype=torch.float64, device=cuda).index_add_(0, tc, dO), 1e-5)
    ident = torch.arange(T, dtype=torch.int32, device=cuda)
    dP1, dWe1 = torch.empty(R, N, D, device=cuda), torch.empty(T, R, device=cuda)
    ds1 = torch.empty(N, D, device=cuda) if dsum else None
    ops.tail_seg_reduce(tptr, ident, W.float(), dO.float(), P.float(), dP1, dWe1, dsum=ds1)
    assert torch.equal(dP, dP1)
    if dsum:
        assert torch.equal(ds, ds1)
    if T:
        assert _maxrel(dWe, dWe1) <= 1e-6


@pytest.mark.parametrize("D,mode", [(256, "split"), (256, "bf16x3"), (256, "exact"), (64, "exact")])
def test_gemm_tn_batched(D, mode, cuda):
    """iddgcn_gemm_tn_batched_f32 (one launch, blockIdx.y = entry, at D = 256 split / bf16x3; the single-call kernels in
    turn otherwise) against float64 references and the single-call results: entries of different row counts
    (one empty), accumulate on / off, up to TN_BATCH entries; the batched launch is deterministic."""
    g = torch.Generator().manual_seed(D + len(mode))
    Ms = [30_001, 4_100, 0, 777]
    ents, refs, singles = [], [], []
    for k, M in enumerate(Ms):
        A = torch.randn(M, D, generator=g, dtype=torch.float64)
        B = torch.randn(M, D, generator=g, dtype=torch.float64) * 10 ** (-3 * k)
        C0 = torch.randn(D, D, generator=g, dtype=torch.float64)
        acc = k % 2 == 1
        Af, Bf = A.float().to(cuda), B.float().to(cuda)
        C = C0.float().to(cuda)
        ents.append((Af, Bf, C, acc))
        refs.append(A.t() @ B + (C0.float().double() if acc else 0))
        Cs = C0.float().to(cuda)
        if M:                                  # (the single-call entry takes no empty operands)
            slab1 = torch.empty(ops.tn_blocks(M, D) * D * D, device=cuda)
            ops.gemm_tn(Af, Bf, Cs, slab1, accumulate=acc, precision=mode)
        singles.append(Cs)
    Cinit = [c.clone() for _, _, c, _ in ents]
    slab = torch.empty(256 * D * D, device=cuda)
    ops.gemm_tn_batched(ents, slab, precision=mode)
    again = [c.clone() for c in Cinit]
    ops.gemm_tn_batched([(a, b, c2, acc) for (a, b, _, acc), c2 in zip(ents, again)], slab, precision=mode)
    for (_, _, C, _), C2, ref, Cs, M in zip(ents, again, refs, singles, Ms):
        assert torch.equal(C, C2)
        ref = ref.to(cuda)
        if M == 0:
            assert torch.equal(C.double(), ref)
            continue
        bar = max(2 * _maxrel(Cs, ref), 2e-6)
        assert _maxrel(C, ref) <= bar


@pytest.mark.parametrize("D", DIMS)
def test_rowgemm_f32_4chain_accumulation(D, cuda):
    """IDDGCN_GEMM_F32_4CHAIN ("exact4", the node-level projections P_r^l = AE_r K_r^l in the exact mode): the
    f32 MFMA products with the k-accumulation in four interleaved fp32 chains summed pairwise.  On
    projection-shaped operands (rows like AE_r = sums of ~20 U[0,1) entity rows, weights N(0, 1): |C| up
    to ~1e3) its error against fp64 is below the single 256-long chain's, the result is deterministic, the
    plain / transposed / accumulate forms all take it, and the D = 256 forms it does not cover are refused."""
    g = torch.Generator().manual_seed(5 * D)
    M = 20_011
    A = (torch.rand(M, D, generator=g, dtype=torch.float64) * 20 + torch.rand(M, 1, generator=g, dtype=torch.float64)).to(cuda)
    B = torch.randn(D, D, generator=g, dtype=torch.float64).to(cuda)
    C0 = torch.randn(M, D, generator=g, dtype=torch.float64).to(cuda) * 100
    for kw, ref in ((dict(), A @ B), (dict(b_trans=True), A @ B.t()), (dict(accumulate=True), C0 + A @ B)):
        errs = {}
        for prec in ("exact", "exact4"):
            C = C0.float().clone() if kw.get("accumulate") else torch.empty(M, D, device=cuda)
            ops.rowgemm(A.float(), B.float(), C, precision=prec, **kw)
            errs[prec] = (C.double() - ref).abs().max().item()
            if prec == "exact4":
                C2 = C0.float().clone() if kw.get("accumulate") else torch.empty(M, D, device=cuda)
                ops.rowgemm(A.float(), B.float(), C2, precision=prec, **kw)
                assert torch.equal(C, C2)
                if D == 256:
                    assert ops.rowgemm_kernel_id(A.float(), B.float(), C, precision=prec, **kw) == 4300
        assert errs["exact4"] <= errs["exact"], (kw, errs)
        assert errs["exact4"] <= 2e-6 * ref.abs().max().item() * np.sqrt(D / 64), (kw, errs)
    if D == 256:       # coefficients / sigma' epilogues keep the single chain at D = 256
        with pytest.raises(L.IddgcnError):
            ops.rowgemm(A.float(), B.float(), torch.empty(M, D, device=cuda), precision="exact4", act=L.ACT_DSIGMOID,
                        aux=torch.rand(M, D, device=cuda))


@pytest.mark.parametrize("R", [2, 5, 8])
def test_engine_projection_batches_cover_every_entry(R, cuda, monkeypatch):
    """The engine's forward hands every node-level projection (3R + 1 of them) to rowgemm_batched in chunks of at
    most L.ROWGEMM_BATCH, each exactly once (a chunk sliced shorter than its stride once left config 5's layer-3
    tables uncomputed)."""
    from iddgcn_amd.engine import Engine, FlatParams
    from iddgcn_amd.graph import get_adj_mats
    from iddgcn_amd.utils import synthetic_graph
    N, D = 300, 256
    pos, neg = synthetic_graph(N, R, 3000, seed=R)
    eng = Engine(N, R, D, cuda, features="bf16" if R == 8 else "f32")
    P = FlatParams(N, R, D, cuda)
    rng = np.random.default_rng(R)
    P.load({name: rng.standard_normal(shape).astype(np.float32) * 0.05 for name, shape, _ in P.layout})
    seen = []
    orig = ops.rowgemm_batched

    def spy(calls):
        assert len(calls) <= L.ROWGEMM_BATCH
        seen.extend(C.data_ptr() for _, _, C, _ in calls)
        return orig(calls)

    monkeypatch.setattr(ops, "rowgemm_batched", spy)
    eng.predict(P, eng.adjacency(get_adj_mats(pos, N, R)), eng.edges(np.concatenate([pos, neg]),
                                                                     np.zeros(len(pos) + len(neg))))
    assert len(seen) == 3 * R + 1 and len(set(seen)) == 3 * R + 1
