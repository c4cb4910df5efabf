"""The fused sigma' backward + dS TN pass over fp32 edge tables in the bf16x3 mode (iddgcn_sigma_tn_f32, ABI 12;
the headline's layer-2/3 edge backward, IDDGCN.py:62-63,79), against the two kernels it replaces and fp64.

Bars:
  * dX (written over X) bitwise equal to the bf16x3 row GEMM's sigma' output (rowgemm256_b3_kernel<0, true>: the
    same six MFMA products in the same order, the same epilogue; x rebuilt exactly from its three bf16 pieces);
  * dS = X^T dO within max(1.25 x the exact-f32 TN's error, 1e-6) of max|ref| of the fp64 product — the bar of the
    two-kernel bf16x3 TN (test_gpu_kernels.py::test_gemm_tn_bf16x3_vs_fp64);
  * deterministic run to run; dS overwritten (a NaN-filled slab / output never leaks in); M = 0 gives dS = 0.
"""
import pytest
import torch

from iddgcn_amd import _lib as L
from iddgcn_amd import ops

pytestmark = pytest.mark.gpu
D = 256


def _maxrel(got, ref):
    return (got.double() - ref).abs().max().item() / max(ref.abs().max().item(), 1e-300)


def _operands(M, kind, g):
    X = torch.rand(M, D, generator=g, dtype=torch.float64)           # sigmoid outputs in (0, 1)
    dO = torch.randn(M, D, generator=g, dtype=torch.float64) * 1e-6
    if kind == "decades":
        dO = dO * 10 ** (6 * torch.rand(M, 1, generator=g, dtype=torch.float64) - 3)
    elif kind == "zero_blocks":
        dO[: M // 2] = 0
        X[M // 3: M // 2] = 0
    S = torch.randn(D, D, generator=g, dtype=torch.float64) / 16
    return X.float(), dO.float(), S.float()


@pytest.mark.parametrize("kind", ["plain", "decades", "zero_blocks"])
@pytest.mark.parametrize("M", [1, 31, 33, 4097, 300_017])
def test_sigma_tn_b3_vs_two_kernels_and_fp64(M, kind, cuda):
    g = torch.Generator().manual_seed(M * 7 + len(kind))
    X, dO, S = (t.to(cuda) for t in _operands(M, kind, g))
    ref_S = X.double().t() @ dO.double()
    # the two kernels the pass replaces: the exact / bf16x3 TN for the bar, the bf16x3 sigma' row GEMM for dX
    slab_tn = torch.empty(ops.tn_blocks(M, D) * D * D, device=cuda)
    errs = {}
    for gm in ("exact", "bf16x3"):
        C = torch.empty(D, D, device=cuda)
        ops.gemm_tn(X, dO, C, slab_tn, precision=gm)
        errs[gm] = _maxrel(C, ref_S)
    dX_ref = torch.empty(M, D, device=cuda)
    ops.rowgemm(dO, S, dX_ref, b_trans=True, act=L.ACT_DSIGMOID, aux=X, precision="bf16x3")

    slab = torch.full((ops.sigma_tn_slab_floats(M),), float("nan"), device=cuda)
    outs = []
    for _ in range(2):
        dS = torch.full((D, D), float("nan"), device=cuda)
        Xi = X.clone()
        ops.sigma_tn(dO, Xi, S, dS, slab, precision="bf16x3")
        outs.append((dS, Xi))
    torch.cuda.synchronize()
    (dS, Xi), (dS2, Xi2) = outs
    assert torch.equal(dS, dS2) and torch.equal(Xi, Xi2), "not deterministic"
    assert torch.equal(Xi, dX_ref), (Xi - dX_ref).abs().max().item()
    err = _maxrel(dS, ref_S)
    assert err <= max(1.25 * errs["exact"], 1e-6), (err, errs)


def test_sigma_tn_b3_empty_and_refusals(cuda):
    S = torch.randn(D, D, device=cuda)
    X = torch.empty(0, D, device=cuda)
    dS = torch.full((D, D), float("nan"), device=cuda)
    slab = torch.empty(ops.sigma_tn_slab_floats(0), device=cuda)
    ops.sigma_tn(X.clone(), X, S, dS, slab, precision="bf16x3")
    torch.cuda.synchronize()
    assert torch.equal(dS, torch.zeros_like(dS))
    # fp32 tables take the bf16x3 form only; a typo'd precision is refused by name
    Xs = torch.rand(64, D, device=cuda)
    for bad in ("exact", "split", "bf16"):
        with pytest.raises(L.IddgcnError):
            ops.sigma_tn(Xs.clone(), Xs, S, dS, slab, precision=bad)
    with pytest.raises(L.IddgcnError):
        ops.sigma_tn(Xs.clone(), Xs, S, dS, slab, precision="bf16x4")
