"""Thin torch-facing wrappers over the C-ABI (one call = one library entry point).

torch is used only as the device-memory / stream provider: every wrapper takes
CUDA(HIP) tensors, validates shapes/dtypes on the host (so a bad shape never
reaches a kernel), and passes raw pointers plus torch's current stream.
Index VALUES (entity / relation ids) are validated where they enter the
product path — graph.get_adj_mats / DeviceAdjacency / ScoredEdges (host or
device build, error flag) and the layer-level calls in model.py; direct callers
of these wrappers can turn on per-call range checks with IDDGCN_CHECK_INDICES=1.
"""
import ctypes
import os

import torch

from . import _lib as L

_F32 = torch.float32
_BF16 = torch.bfloat16
_I32 = torch.int32


def _ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


_PRECISION = {"exact": L.GEMM_EXACT_F32, "split": L.GEMM_SPLIT_F16, "exact4": L.GEMM_F32_4CHAIN,
              "bf16x3": L.GEMM_BF16X3, "bf16": L.GEMM_BF16,
              L.GEMM_EXACT_F32: L.GEMM_EXACT_F32, L.GEMM_SPLIT_F16: L.GEMM_SPLIT_F16,
              L.GEMM_F32_4CHAIN: L.GEMM_F32_4CHAIN, L.GEMM_BF16X3: L.GEMM_BF16X3, L.GEMM_BF16: L.GEMM_BF16}


def _prec(precision):
    """GEMM operand precision of one call (include/iddgcn.h IDDGCN_GEMM_*): "exact" / "split" / "exact4" (f32
    MFMA with four interleaved accumulation chains: row GEMMs, plain form at D = 256) / "bf16x3" (every fp32
    operand split exactly into three bf16 pieces, six bf16 MFMA products, fp32 accumulation) / "bf16" (bf16 edge
    tables only: every MFMA operand rounded to bf16, one product per term) or the constant."""
    if precision not in _PRECISION:
        raise L.IddgcnError(f"precision must be 'exact', 'split', 'exact4', 'bf16x3' or 'bf16', got {precision!r}")
    return _PRECISION[precision]


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _req(t, dtype, shape=None, name="tensor"):
    if t is None:
        return
    if not t.is_cuda:
        raise L.IddgcnError(f"{name} must be a GPU tensor (no CPU fallback)")
    if t.dtype != dtype:
        raise L.IddgcnError(f"{name}: expected {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise L.IddgcnError(f"{name} must be contiguous")
    if shape is not None and tuple(t.shape) != tuple(shape):
        raise L.IddgcnError(f"{name}: expected shape {tuple(shape)}, got {tuple(t.shape)}")


# Index RANGES are checked here only when IDDGCN_CHECK_INDICES=1 (one device reduction + host sync per
# index array, a debug mode): the product path's indices come from graph.ScoredEdges / DeviceAdjacency,
# whose builders validate every entity / relation id on the host or in the device build (error flag).
CHECK_INDEX_RANGES = os.environ.get("IDDGCN_CHECK_INDICES", "0") == "1"


def _idx_ok(idx, n_rows, bound, name):
    """dtype / shape / contiguity of an int32 index array; with CHECK_INDEX_RANGES (or always for a
    CPU-resident check-free size-0 array) also 0 <= idx < bound."""
    if idx is None:
        return
    _req(idx, _I32, (n_rows,), name)
    if CHECK_INDEX_RANGES and bound is not None and idx.numel():
        lo, hi = int(idx.min()), int(idx.max())
        if lo < 0 or hi >= int(bound):
            raise L.IddgcnError(f"{name}: index out of range [0, {int(bound)}): min {lo}, max {hi}")


def spmm_csr(row_ptr, col, vals, X, Y, n_seg, n_rows, accumulate=False):
    D = X.shape[1]
    _req(row_ptr, _I32, (n_seg * (n_rows + 1),), "row_ptr")
    _req(col, _I32, None, "col")
    _req(vals, _F32, None, "vals")
    _req(X, _F32, None, "X")
    _req(Y, _F32, (n_seg, n_rows, D), "Y")
    L.check(L.lib().iddgcn_spmm_csr_f32(_stream(), n_seg, n_rows, D, _ptr(row_ptr), _ptr(col), _ptr(vals),
                                        _ptr(X), _ptr(Y), int(accumulate)), "spmm_csr")


def sddmm_csr(row_ptr, col, G, X, out, n_seg, n_rows):
    """out[k] = <G[s][row(k)], X[col[k]]> over the batched CSR (gradient w.r.t. adjacency values)."""
    D = X.shape[1]
    _req(row_ptr, _I32, (n_seg * (n_rows + 1),), "row_ptr")
    _req(col, _I32, None, "col")
    _req(G, _F32, (n_seg, n_rows, D), "G")
    _req(X, _F32, None, "X")
    _req(out, _F32, (col.shape[0],), "out")
    L.check(L.lib().iddgcn_sddmm_csr_f32(_stream(), n_seg, n_rows, D, _ptr(row_ptr), _ptr(col), _ptr(G), _ptr(X),
                                         _ptr(out)), "sddmm_csr")


def rowgemm(A, B, C, **kw):
    """C = epilogue(A[a_idx] · B^(T)) (include/iddgcn.h, iddgcn_rowgemm_f32); see _rowgemm_args.  bf16 A
    (the bf16-feature mode's edge tables) selects iddgcn_rowgemm_bf16: A, aux and C are then bf16."""
    args = _rowgemm_args(A, B, C, **kw)
    if A.dtype == _BF16:
        L.check(L.lib().iddgcn_rowgemm_bf16(_stream(), ctypes.byref(args)), "rowgemm_bf16")
    else:
        L.check(L.lib().iddgcn_rowgemm_f32(_stream(), ctypes.byref(args)), "rowgemm")


def rowgemm_kernel_id(A, B, C, **kw):
    """Which kernel rowgemm(A, B, C, **kw) runs (iddgcn_rowgemm_kernel_id): 300 + 10*NV + ... (+2000 split
    operands) for the D=256 v3 pipeline, 100 the register-staged one."""
    args = _rowgemm_args(A, B, C, **kw)
    return int(L.lib().iddgcn_rowgemm_kernel_id(ctypes.byref(args)))


def rowgemm_batched(calls):
    """Independent row GEMMs of one width in one launch (iddgcn_rowgemm_batched_f32).  calls: list of
    (A, B, C, kwargs) as for rowgemm; at most L.ROWGEMM_BATCH (25)."""
    if not calls:
        return
    arr = (L.RowGemmArgs * len(calls))(*[_rowgemm_args(A, B, C, **kw) for A, B, C, kw in calls])
    L.check(L.lib().iddgcn_rowgemm_batched_f32(_stream(), arr, len(calls)), "rowgemm_batched")


def _rowgemm_args(A, B, C, *, a_idx=None, b_trans=False, accumulate=False, coef=None, coef_idx=None, V=None,
                  v_idx=None, v_rel_stride=0, v_row_stride=None, act=L.ACT_NONE, aux=None, M=None, planes=0,
                  precision="exact"):
    """C = epilogue(A[a_idx] · B^(T)) (include/iddgcn.h, iddgcn_rowgemm_f32).  planes: L.PLANES_* flags,
    which of A / C / aux are pre-split planes tables (fp32-shaped tensors holding [hi | lo] fp16 rows;
    D = 256, split GEMM mode).  precision, per call: "exact" (v_mfma_f32_32x32x2_f32, bitwise an fmaf chain),
    "exact4" (the same MFMA, four interleaved accumulation chains: the node-level projections), "bf16x3" (fp32
    operands split exactly into three bf16 pieces, six bf16 MFMA products, fp32 accumulation) or "split"
    (split-fp16 operands, 22 significant bits); D < 256 runs exact f32 in every mode."""
    D = B.shape[0]
    M = C.shape[0] if M is None else M
    R = 0 if coef is None else coef.shape[-1]
    et = A.dtype if A.dtype == _BF16 else _F32         # edge-table element type (A, C, aux)
    _req(A, et, None, "A")
    _req(B, _F32, (D, D), "B")
    _req(C, et, (M, D), "C")
    if A.dim() != 2 or A.shape[1] != D:
        raise L.IddgcnError(f"A must be (rows, {D})")
    if a_idx is None and A.shape[0] < M:
        raise L.IddgcnError("A has fewer rows than C")
    _idx_ok(a_idx, M, A.shape[0], "a_idx")
    if R:
        _req(coef, _F32, None, "coef")
        _req(V, _F32, None, "V")
        _idx_ok(coef_idx, M, coef.shape[0], "coef_idx")
        vrows = (int(v_rel_stride) // int(D if v_row_stride is None else v_row_stride)
                 if (v_row_stride is None or v_row_stride) and v_rel_stride else None)
        _idx_ok(v_idx, M, vrows, "v_idx")
    if act == L.ACT_DSIGMOID:
        _req(aux, et, (M, D), "aux")
    return L.RowGemmArgs(
        M=M, D=D, A=_ptr(A), a_idx=_ptr(a_idx), B=_ptr(B), b_trans=int(b_trans), C=_ptr(C),
        accumulate=int(accumulate), R=R, coef=_ptr(coef), coef_idx=_ptr(coef_idx), V=_ptr(V),
        v_idx=_ptr(v_idx), v_rel_stride=int(v_rel_stride),
        v_row_stride=int(D if v_row_stride is None else v_row_stride), act=int(act), aux=_ptr(aux),
        planes=int(planes), precision=_prec(precision))


def tn_blocks(M, D):
    return int(L.lib().iddgcn_gemm_tn_blocks(int(M), int(D)))


def _tn_prec(precision):
    """Operand precision of a TN GEMM: "exact", "bf16x3" or "split" (include/iddgcn.h; the TN kernels take no
    four-chain form, so "exact4" is refused here rather than by the C side's IDDGCN_E_BAD_ARG)."""
    if precision in ("exact4", "bf16", L.GEMM_F32_4CHAIN, L.GEMM_BF16):
        raise L.IddgcnError(f"gemm_tn: precision {precision!r} is a row-GEMM form; use 'exact', 'bf16x3' or 'split'")
    return _prec(precision)


def gemm_tn(A, B, C, slab, accumulate=False, a_planes=False, precision="exact"):
    """C (+)= A^T B; bf16 A and B (the bf16-feature mode) select iddgcn_gemm_tn_bf16; a_planes: A is a
    pre-split planes table (iddgcn_gemm_tn_planes_f32, D = 256, split GEMM mode); precision: the fp32 form's
    operand precision ("exact", "bf16x3" or "split" at D = 256; other widths exact f32)."""
    prec = _tn_prec(precision)
    M, D = A.shape
    et = _BF16 if A.dtype == _BF16 else _F32
    _req(A, et, (M, D), "A")
    _req(B, et, (M, D), "B")
    _req(C, _F32, (D, D), "C")
    nb = tn_blocks(M, D)
    if slab.numel() < nb * D * D:
        raise L.IddgcnError("gemm_tn slab too small")
    args = (_stream(), M, D, _ptr(A), _ptr(B), _ptr(slab), nb, _ptr(C), int(accumulate))
    if a_planes:
        if et != _F32 or prec != L.GEMM_SPLIT_F16:
            raise L.IddgcnError("gemm_tn: planes A takes an fp32-shaped table in the split mode")
        rc = L.lib().iddgcn_gemm_tn_planes_f32(*args)
    elif et == _BF16:
        rc = L.lib().iddgcn_gemm_tn_bf16(*args)
    else:
        rc = L.lib().iddgcn_gemm_tn_f32(*args, prec)
    L.check(rc, "gemm_tn")


def sigma_tn(dO, X, S, dS, slab, precision="exact"):
    """A layer's edge backward GEMM pair in one pass (the autodiff of IDDGCN.py:62-63,79): dS = X^T dO (overwritten)
    and X = (dO S^T) * X (1 - X) in place.
      * bf16 tables (iddgcn_sigma_tn_bf16, ABI 11): the weights as a bf16 hi + lo pair ("exact", "split", "bf16x3"),
        or rounded to bf16 ("bf16", as rowgemm's bf16 form);
      * fp32 tables (iddgcn_sigma_tn_f32, ABI 12): precision "bf16x3" only (every operand split exactly into three
        bf16 pieces; X bitwise the bf16x3 row GEMM's sigma' output)."""
    M, D = X.shape
    prec = _prec(precision)
    et = _BF16 if X.dtype == _BF16 else _F32
    _req(X, et, (M, D), "X")
    _req(dO, et, (M, D), "dO")
    _req(S, _F32, (D, D), "S")
    _req(dS, _F32, (D, D), "dS")
    _req(slab, _F32, None, "slab")
    if et == _BF16:
        if prec not in (L.GEMM_EXACT_F32, L.GEMM_SPLIT_F16, L.GEMM_BF16X3, L.GEMM_BF16):
            raise L.IddgcnError(f"sigma_tn: precision {precision!r} is not a form of the bf16 pass")
        rc = L.lib().iddgcn_sigma_tn_bf16(_stream(), M, D, _ptr(dO), _ptr(X), _ptr(S), _ptr(slab), slab.numel(),
                                          _ptr(dS), prec)
    else:
        if prec != L.GEMM_BF16X3:
            raise L.IddgcnError(f"sigma_tn: fp32 tables take precision 'bf16x3' only, got {precision!r}")
        rc = L.lib().iddgcn_sigma_tn_f32(_stream(), M, D, _ptr(dO), _ptr(X), _ptr(S), _ptr(slab), slab.numel(),
                                         _ptr(dS), prec)
    L.check(rc, "sigma_tn")


def sigma_tn_slab_floats(M, D=256):
    return int(L.lib().iddgcn_sigma_tn_ranges(M)) * D * D


def gemm_tn_batched(entries, slab, precision="exact"):
    """Up to L.TN_BATCH independent C (+)= A^T B, entries = [(A, B, C, accumulate), ...] (fp32, same D), in one
    launch (iddgcn_gemm_tn_batched_f32, ABI 5; one launch at D = 256 in the split and bf16x3 modes); slab holds
    the partials of all entries.  precision: as gemm_tn."""
    prec = _tn_prec(precision)
    if not entries:
        return
    if len(entries) > L.TN_BATCH:
        raise L.IddgcnError(f"gemm_tn_batched: at most {L.TN_BATCH} entries")
    D = entries[0][0].shape[1]
    arr = (L.TnArgs * len(entries))()
    for k, (A, B, C, acc) in enumerate(entries):
        M = A.shape[0]
        _req(A, _F32, (M, D), "A")
        _req(B, _F32, (M, D), "B")
        _req(C, _F32, (D, D), "C")
        arr[k] = L.TnArgs(M, _ptr(A), _ptr(B), _ptr(C), int(bool(acc)))
    _req(slab, _F32, None, "slab")
    L.check(L.lib().iddgcn_gemm_tn_batched_f32(_stream(), D, arr, len(entries), _ptr(slab), slab.numel(), prec),
            "gemm_tn_batched")


def tn_narrow_blocks(M):
    return int(L.lib().iddgcn_gemm_tn_narrow_blocks(int(M)))


def gemm_tn_narrow(A, dz, dWa, dba, slab, accumulate=False):
    M, D = A.shape
    R = dz.shape[1]
    _req(dz, _F32, (M, R), "dz")
    _req(dWa, _F32, (D, R), "dWa")
    _req(dba, _F32, (R,), "dba")
    nb = tn_narrow_blocks(M)
    if slab.numel() < (nb + 1) * (D + 1) * R:
        raise L.IddgcnError("gemm_tn_narrow slab too small")
    L.check(L.lib().iddgcn_gemm_tn_narrow_f32(_stream(), M, D, R, _ptr(A), _ptr(dz), _ptr(slab), nb, _ptr(dWa),
                                              _ptr(dba), int(accumulate)), "gemm_tn_narrow")


def alpha_fwd(X, Wa, ba, S_out, W_out, x_idx=None, M=None):
    D, R = Wa.shape
    M = S_out.shape[0] if M is None else M
    _req(X, _F32, None, "X")
    _req(Wa, _F32, (D, R), "W_alpha")
    _req(ba, _F32, (R,), "b_alpha")
    _req(S_out, _F32, (M, R), "S_out")
    _req(W_out, _F32, (M, R), "W_out")
    _idx_ok(x_idx, M, X.shape[0], "x_idx")
    L.check(L.lib().iddgcn_alpha_fwd_f32(_stream(), M, D, R, _ptr(X), _ptr(x_idx), _ptr(Wa), _ptr(ba),
                                         _ptr(S_out), _ptr(W_out)), "alpha_fwd")


def combine(Y, coef, V, out, *, y_idx=None, coef_idx=None, v_idx=None, v_rel_stride=None, planes_out=False):
    """out = sigmoid(Y[y_idx] + sum_r coef[coef_idx, r] V_r[v_idx]) (iddgcn_combine_f32).  A bf16 out (the
    bf16-feature mode) or planes_out (out a pre-split planes table, D = 256) take the run form:
    y_idx and v_idx the same array, per-row coefficients."""
    M, D = out.shape
    R = coef.shape[-1]
    if out.dtype == _BF16 or planes_out:
        if y_idx is None or v_idx is not y_idx or coef_idx is not None:
            raise L.IddgcnError("combine into bf16 / planes: y_idx and v_idx must be the same array, no coef_idx")
        _req(out, _BF16 if out.dtype == _BF16 else _F32, (M, D), "out")
        _req(Y, _F32, None, "Y")
        _req(coef, _F32, (M, R), "coef")
        _idx_ok(y_idx, M, Y.shape[0], "y_idx")
        vrs = V.shape[1] * D if v_rel_stride is None else v_rel_stride
        fn = L.lib().iddgcn_combine_bf16 if out.dtype == _BF16 else L.lib().iddgcn_combine_planes_f32
        L.check(fn(_stream(), M, D, R, _ptr(Y), _ptr(y_idx), _ptr(coef), _ptr(V), int(vrs), _ptr(out)), "combine_run")
        return
    _req(Y, _F32, None, "Y")
    _req(coef, _F32, None, "coef")
    _req(V, _F32, None, "V")
    _req(out, _F32, (M, D), "out")
    vrs = V.shape[1] * D if v_rel_stride is None else v_rel_stride
    for n, ix, bound in (("y_idx", y_idx, Y.shape[0]), ("coef_idx", coef_idx, coef.shape[0]),
                         ("v_idx", v_idx, int(vrs) // D)):
        _idx_ok(ix, M, bound, n)
    L.check(L.lib().iddgcn_combine_f32(_stream(), M, D, R, _ptr(Y), _ptr(y_idx), _ptr(coef), _ptr(coef_idx),
                                       _ptr(V), _ptr(v_idx), int(vrs), _ptr(out)), "combine")


def distmult_blocks(T):
    return int(L.lib().iddgcn_distmult_blocks(int(T)))


def distmult_bce(Xh, h_idx, Xt, r_idx, rel, *, t_idx=None, y=None, scale=1.0, p_out=None, s_out=None, ds_out=None,
                 do_out=None, drel_slab=None, loss_slab=None):
    """DistMult score (IDDGCN.py:103-109): p_out = sigmoid(s), s_out = s (the pre-sigmoid logit); with y the
    Keras BCE and both backward seeds."""
    T = h_idx.shape[0]
    R, D = rel.shape
    _req(h_idx, _I32, (T,), "h_idx")
    _req(r_idx, _I32, (T,), "r_idx")
    bf = Xt.dtype == _BF16
    _req(Xh, _F32, None, "Xh")
    _req(Xt, _BF16 if bf else _F32, None, "Xt")
    _req(rel, _F32, (R, D), "rel")
    _req(y, _F32, (T,), "y")
    _req(p_out, _F32, (T,), "p_out")
    _req(s_out, _F32, (T,), "s_out")
    _idx_ok(h_idx, T, Xh.shape[0], "h_idx")
    _idx_ok(t_idx, T, Xt.shape[0], "t_idx")
    _idx_ok(r_idx, T, R, "r_idx")
    if t_idx is None and Xt.shape[0] < T:
        raise L.IddgcnError("distmult: Xt has fewer rows than scored edges")
    nb = distmult_blocks(T)
    if y is not None:
        _req(ds_out, _F32, (T,), "ds_out")
        _req(do_out, Xt.dtype, (T, D), "do_out")
        if drel_slab.numel() < nb * R * D or loss_slab.numel() < nb:
            raise L.IddgcnError("distmult slabs too small")
    fn = L.lib().iddgcn_distmult_bce_bf16 if bf else L.lib().iddgcn_distmult_bce_f32
    L.check(fn(_stream(), T, D, R, _ptr(Xh), _ptr(h_idx), _ptr(Xt), _ptr(t_idx),
                                            _ptr(r_idx), _ptr(rel), _ptr(y), float(scale), _ptr(p_out),
                                            _ptr(s_out), _ptr(ds_out), _ptr(do_out), _ptr(drel_slab), _ptr(loss_slab),
                                            nb),
            "distmult_bce")
    return nb


def distmult_bce_heads(seg_ptr, perm, Xh, Xt, r_idx, rel, y, do_out, dXh, drel_slab, loss_slab, *, scale=1.0,
                      p_out=None, s_out=None, ds_out=None):
    """Training DistMult + BCE + tail seed (do_out) + head seed (dXh) in one pass over head segments.
    y=None selects the prediction seed (gradient of scale * sum_e p_e; loss slabs sum p_e)."""
    T = r_idx.shape[0]
    n_nodes, D = dXh.shape
    R = rel.shape[0]
    _req(seg_ptr, _I32, (n_nodes + 1,), "seg_ptr")
    _req(perm, _I32, (T,), "perm")
    _req(r_idx, _I32, (T,), "r_idx")
    et = _BF16 if Xt.dtype == _BF16 else _F32
    _req(Xh, _F32, (n_nodes, D), "Xh")
    _req(Xt, et, (T, D), "Xt")
    _req(rel, _F32, (R, D), "rel")
    _req(y, _F32, (T,), "y")
    _req(do_out, et, (T, D), "do_out")
    _req(dXh, _F32, (n_nodes, D), "dXh")
    _req(p_out, _F32, (T,), "p_out")
    _req(s_out, _F32, (T,), "s_out")
    _req(ds_out, _F32, (T,), "ds_out")
    nb = distmult_blocks(T)
    if drel_slab.numel() < nb * R * D or loss_slab.numel() < nb:
        raise L.IddgcnError("distmult slabs too small")
    fn = L.lib().iddgcn_distmult_bce_heads_bf16 if et == _BF16 else L.lib().iddgcn_distmult_bce_heads_f32
    L.check(fn(_stream(), n_nodes, D, R, _ptr(seg_ptr), _ptr(perm), _ptr(Xh),
                                                  _ptr(Xt), _ptr(r_idx), _ptr(rel), _ptr(y), float(scale),
                                                  _ptr(p_out), _ptr(s_out), _ptr(ds_out), _ptr(do_out), _ptr(dXh),
                                                  _ptr(drel_slab), _ptr(loss_slab), nb), "distmult_bce_heads")
    return nb


def seg_gather_reduce(seg_ptr, rows, out, *, perm=None, coef=None, r_idx=None, rel=None, X=None):
    n_nodes, D = out.shape
    _req(seg_ptr, _I32, (n_nodes + 1,), "seg_ptr")
    _req(out, _F32, (n_nodes, D), "out")
    L.check(L.lib().iddgcn_seg_gather_reduce_f32(_stream(), n_nodes, D, _ptr(seg_ptr), _ptr(perm), _ptr(coef),
                                                 _ptr(r_idx), _ptr(rel), _ptr(rows), _ptr(X), _ptr(out)),
            "seg_gather_reduce")


def _req_rel_rows(t, shape, name):
    """An (R, n, D) fp32 GPU view whose rows are contiguous (a node-row range of an (R, N, D) table keeps its
    relation stride); returns that stride (elements)."""
    if t is None:
        return 0
    if not t.is_cuda or t.dtype != _F32:
        raise L.IddgcnError(f"{name} must be an fp32 GPU tensor (no CPU fallback)")
    if tuple(t.shape) != tuple(shape) or t.stride(1) != shape[2] or t.stride(2) != 1:
        raise L.IddgcnError(f"{name} must be {tuple(shape)} with contiguous rows")
    return t.stride(0)


def tail_seg_reduce_head(seg_ptr, W, dO, P, dP, dWedge, head_dO, Wn, dwh, dsum=None):
    """tail_seg_reduce with per-edge W on bf16 rows at R = 8, D = 256, fused with the head chain's node terms of the
    same layer (iddgcn_tail_seg_reduce_head_bf16, ABI 9): dP[r][n] = tail sum + Wn[n][r] head_dO[n], dsum[n] = tail
    sum + head_dO[n], dwh[n][r] = <head_dO[n], P_r[n]>; the head backward is then head_dz.  P, dP: (R, n, D) views
    with contiguous rows (a node-row range: seg_ptr the matching slice of the tail pointers, absolute edge offsets)."""
    R, n_nodes, D = P.shape
    _req(seg_ptr, _I32, (n_nodes + 1,), "seg_ptr")
    ps = _req_rel_rows(P, (R, n_nodes, D), "P")
    dps = _req_rel_rows(dP, (R, n_nodes, D), "dP")
    _req(dsum, _F32, (n_nodes, D), "dsum")
    _req(head_dO, _F32, (n_nodes, D), "head_dO")
    _req(Wn, _F32, (n_nodes, R), "Wn")
    _req(dwh, _F32, (n_nodes, R), "dwh")
    _req(dO, _BF16, None, "dO")
    if W.shape[0] != dO.shape[0]:
        raise L.IddgcnError("tail_seg_reduce_head: per-edge W must have one row per edge")
    L.check(L.lib().iddgcn_tail_seg_reduce_head_bf16(_stream(), n_nodes, D, R, _ptr(seg_ptr), _ptr(W), _ptr(dO),
                                                     _ptr(P), ps, _ptr(dP), dps, _ptr(dsum),
                                                     _ptr(dWedge), _ptr(head_dO), _ptr(Wn), _ptr(dwh)),
            "tail_seg_reduce_head")


def head_dz(Ssm, W, hseg_ptr, hperm, dWedge, dwh, dz):
    """The head backward after tail_seg_reduce_head (iddgcn_head_dz_f32, ABI 9): dW_r = dwh[n][r] + the head
    segment's dWedge rows, then the softmax-sigmoid backward into dz (n, R)."""
    n_nodes, R = dz.shape
    for t, nm in ((Ssm, "Ssm"), (W, "W"), (dwh, "dwh"), (dz, "dz")):
        _req(t, _F32, (n_nodes, R), nm)
    _req(hseg_ptr, _I32, (n_nodes + 1,), "hseg_ptr")
    _req(hperm, _I32, None, "hperm")
    _req(dWedge, _F32, None, "dWedge")
    L.check(L.lib().iddgcn_head_dz_f32(_stream(), n_nodes, R, _ptr(Ssm), _ptr(W), _ptr(hseg_ptr), _ptr(hperm),
                                       _ptr(dWedge), _ptr(dwh), _ptr(dz)), "head_dz")


def tail_seg_reduce(seg_ptr, h_idx, W, dO, P, dP, dWedge, dsum=None):
    """Tail segment sums of a layer's backward (include/iddgcn.h iddgcn_tail_seg_reduce_*): dP[r][n] = sum over the
    tail segment of n of W[e][r] dO[e], dWedge[e][r] = <dO[e], P_r[t_e]> (and dsum[n] = sum of dO[e]).  P, dP: (R, n,
    D) views with contiguous rows (a node-row range: seg_ptr the matching slice of the tail pointers)."""
    R, n_nodes, D = P.shape
    _req(seg_ptr, _I32, (n_nodes + 1,), "seg_ptr")
    ps = _req_rel_rows(P, (R, n_nodes, D), "P")
    dps = _req_rel_rows(dP, (R, n_nodes, D), "dP")
    _req(dsum, _F32, (n_nodes, D), "dsum")
    if h_idx is None and W.shape[0] != dO.shape[0]:
        raise L.IddgcnError("tail_seg_reduce: per-edge W must have one row per edge")
    _req(dO, _BF16 if dO.dtype == _BF16 else _F32, None, "dO")
    fn = L.lib().iddgcn_tail_seg_reduce_bf16 if dO.dtype == _BF16 else L.lib().iddgcn_tail_seg_reduce_f32
    L.check(fn(_stream(), n_nodes, D, R, _ptr(seg_ptr), _ptr(h_idx), _ptr(W),
                                               _ptr(dO), _ptr(P), ps, _ptr(dP), dps, _ptr(dsum),
                                               _ptr(dWedge)), "tail_seg_reduce")


def head_bwd_node(dO, P, Ssm, W, dP, dz, *, hseg_ptr=None, hperm=None, dWedge=None, dsum=None, ep=None):
    """Head-chain backward of one layer over the rows of dO (include/iddgcn.h iddgcn_head_bwd_node_f32).  P and dP
    are (R, n, D) views whose rows are contiguous (a row range of the (R, N, D) node tables keeps their relation
    stride); ``ep``: (n, R) head sums of dWedge computed elsewhere (node-partitioned steps)."""
    R, n_nodes, D = P.shape
    _req(dO, _F32, (n_nodes, D), "dO")
    _req(Ssm, _F32, (n_nodes, R), "Ssm")
    _req(W, _F32, (n_nodes, R), "W")
    _req(dz, _F32, (n_nodes, R), "dz")
    _req(dsum, _F32, (n_nodes, D), "dsum")
    _req(ep, _F32, (n_nodes, R), "ep")
    for t, nm in ((P, "P"), (dP, "dP")):
        if t is None:             # dP None (ABI 9): its head term was added by tail_seg_reduce_head
            continue
        if tuple(t.shape) != (R, n_nodes, D) or t.stride(1) != D or t.stride(2) != 1:
            raise L.IddgcnError(f"head_bwd_node: {nm} must be (R, n, D) with contiguous rows")
    L.check(L.lib().iddgcn_head_bwd_node_f32(_stream(), n_nodes, D, R, _ptr(dO), _ptr(P), P.stride(0), _ptr(Ssm),
                                             _ptr(W), _ptr(hseg_ptr), _ptr(hperm), _ptr(dWedge), _ptr(ep), _ptr(dP),
                                             dP.stride(0) if dP is not None else 0, _ptr(dsum), _ptr(dz)),
            "head_bwd_node")


def head_wsum(hptr, hperm, w, out):
    """out[n] = sum of w[hperm[k]] over the head segment k in [hptr[n], hptr[n+1]) (iddgcn_head_wsum_f32)."""
    n_nodes, R = out.shape
    _req(out, _F32, (n_nodes, R), "out")
    _req(w, _F32, None, "w")
    if hptr.numel() != n_nodes + 1:
        raise L.IddgcnError("head_wsum: hptr must have n + 1 entries")
    L.check(L.lib().iddgcn_head_wsum_f32(_stream(), n_nodes, R, _ptr(hptr), _ptr(hperm), _ptr(w), _ptr(out)),
            "head_wsum")


def gather_rows(src, idx, dst):
    """dst[e] = src[idx[e]] for narrow rows (src: (N, w), idx: (M,) int32, dst: (M, w))."""
    M, w = dst.shape
    _req(src, _F32, None, "src")
    _req(idx, _I32, (M,), "idx")
    _req(dst, _F32, (M, w), "dst")
    if src.dim() != 2 or src.shape[1] != w:
        raise L.IddgcnError("gather_rows: width mismatch")
    L.check(L.lib().iddgcn_gather_rows_f32(_stream(), M, w, _ptr(src), _ptr(idx), _ptr(dst)), "gather_rows")


def reduce_slabs(slab, n_slabs, out, accumulate=False, scale=1.0):
    n = out.numel()
    L.check(L.lib().iddgcn_reduce_slabs_f32(_stream(), n_slabs, n, _ptr(slab), _ptr(out), int(accumulate),
                                            float(scale)), "reduce_slabs")


def adam(var, m, v, g, alpha, b1, b2, eps, sparse_form):
    n = var.numel()
    for t, nm in ((m, "m"), (v, "v"), (g, "g")):
        if t.numel() != n:
            raise L.IddgcnError(f"adam: {nm} size mismatch")
    L.check(L.lib().iddgcn_adam_f32(_stream(), n, _ptr(var), _ptr(m), _ptr(v), _ptr(g), float(alpha), float(b1),
                                    float(b2), float(eps), int(sparse_form)), "adam")


def adam_table(var, m, v, g, alpha_table, step, b1, b2, eps, sparse_form):
    """iddgcn_adam_f32 with alpha = alpha_table[step[0]] read on the device (graph-replayable)."""
    n = var.numel()
    for t, nm in ((m, "m"), (v, "v"), (g, "g")):
        if t.numel() != n:
            raise L.IddgcnError(f"adam: {nm} size mismatch")
    _req(alpha_table, _F32, None, "alpha_table")
    _req(step, _I32, (1,), "step")
    L.check(L.lib().iddgcn_adam_table_f32(_stream(), n, _ptr(var), _ptr(m), _ptr(v), _ptr(g), _ptr(alpha_table),
                                          _ptr(step), float(b1), float(b2), float(eps), int(sparse_form)),
            "adam_table")


def step_advance(step, loss_history=None, loss=None):
    """loss_history[step] = loss; step += 1 (one device thread)."""
    _req(step, _I32, (1,), "step")
    L.check(L.lib().iddgcn_step_advance(_stream(), _ptr(step), _ptr(loss_history), _ptr(loss)), "step_advance")


# -- device graph build (include/iddgcn_graph.h) ------------------------------------------------
_I64 = torch.int64
_U8 = torch.uint8


def _workspace(nbytes, device):
    if nbytes < 0:
        raise L.IddgcnError("graph build: sizes out of range")
    return torch.empty(max(int(nbytes), 1), dtype=_U8, device=device)


def radix_sort(keys, vals=None, *, end_bit=None, argsort=False):
    """Stable LSD radix sort of int32/int64 keys (non-negative; bits [0, end_bit)).  Returns
    (sorted keys, sorted vals) where vals is `vals` permuted, the stable argsort if argsort=True,
    or None."""
    if keys.dtype not in (_I32, _I64):
        raise L.IddgcnError("radix_sort: keys must be int32 or int64")
    _req(keys, keys.dtype, None, "keys")
    _req(vals, _I32, (keys.shape[0],), "vals")
    kb = keys.element_size()
    n = keys.shape[0]
    end_bit = 8 * kb if end_bit is None else int(end_bit)
    ko = torch.empty_like(keys)
    vo = torch.empty(n, dtype=_I32, device=keys.device) if (vals is not None or argsort) else None
    ws = _workspace(L.lib().iddgcn_radix_sort_workspace(n, kb), keys.device)
    L.check(L.lib().iddgcn_radix_sort_pairs(_stream(), n, kb, end_bit, _ptr(keys), _ptr(vals), _ptr(ko), _ptr(vo),
                                            _ptr(ws), ws.numel()), "radix_sort")
    return ko, vo


def build_adjacency(triples, N, R):
    """utils1.get_adj_mats + DeviceAdjacency's CSR layouts on the GPU.  triples: (M, 3) int64 GPU
    tensor.  Returns a dict of GPU tensors (capacity M + R) and the host counts
    (nnz, placeholders, error)."""
    _req(triples, _I64, None, "triples")
    if triples.dim() != 2 or triples.shape[1] != 3:
        raise L.IddgcnError(f"triples must be (M, 3), got {tuple(triples.shape)}")
    M = triples.shape[0]
    dev = triples.device
    need = L.lib().iddgcn_adjacency_workspace(M, N, R)
    ws = _workspace(need, dev)
    C = M + R
    out = {"fwd_ptr": torch.empty(R * (N + 1), dtype=_I32, device=dev),
           "fwd_col": torch.empty(C, dtype=_I32, device=dev), "fwd_val": torch.empty(C, dtype=_F32, device=dev),
           "bwd_ptr": torch.empty(N + 1, dtype=_I32, device=dev),
           "bwd_col": torch.empty(C, dtype=_I32, device=dev), "bwd_src": torch.empty(C, dtype=_I32, device=dev),
           "bwd_val": torch.empty(C, dtype=_F32, device=dev)}
    counts = torch.empty(3, dtype=_I32, device=dev)
    o = out
    L.check(L.lib().iddgcn_build_adjacency(_stream(), M, N, R, _ptr(triples), _ptr(o["fwd_ptr"]), _ptr(o["fwd_col"]),
                                           _ptr(o["fwd_val"]), _ptr(o["bwd_ptr"]), _ptr(o["bwd_col"]),
                                           _ptr(o["bwd_src"]), _ptr(o["bwd_val"]), _ptr(counts), _ptr(ws),
                                           ws.numel()), "build_adjacency")
    nnz, nph, err = (int(x) for x in counts.cpu())     # the one host synchronisation of the build
    return out, nnz, nph, err


def build_scored_edges(triples, labels, N, R):
    """graph.ScoredEdges on the GPU: tail-sorted (stable) h/r/t, gathered labels, tptr, hperm, hptr,
    inv.  Returns (dict of GPU tensors, error flag)."""
    _req(triples, _I64, None, "triples")
    if triples.dim() != 2 or triples.shape[1] != 3:
        raise L.IddgcnError(f"triples must be (T, 3), got {tuple(triples.shape)}")
    T = triples.shape[0]
    dev = triples.device
    _req(labels, _F32, (T,), "labels")
    ws = _workspace(L.lib().iddgcn_scored_edges_workspace(T, N), dev)
    o = {k: torch.empty(T, dtype=_I32, device=dev) for k in ("h", "r", "t", "hperm")}
    o["y"] = torch.empty(T, dtype=_F32, device=dev) if labels is not None else None
    o["tptr"] = torch.empty(N + 1, dtype=_I32, device=dev)
    o["hptr"] = torch.empty(N + 1, dtype=_I32, device=dev)
    o["inv"] = torch.empty(T, dtype=_I64, device=dev)
    err = torch.empty(1, dtype=_I32, device=dev)
    L.check(L.lib().iddgcn_build_scored_edges(_stream(), T, N, R, _ptr(triples), _ptr(labels), _ptr(o["h"]),
                                              _ptr(o["r"]), _ptr(o["t"]), _ptr(o["y"]), _ptr(o["tptr"]),
                                              _ptr(o["hperm"]), _ptr(o["hptr"]), _ptr(o["inv"]), _ptr(err), _ptr(ws),
                                              ws.numel()), "build_scored_edges")
    return o, int(err.item())


# -- similarity graph (include/iddgcn_similarity.h) ---------------------------------------------
def similarity_pairs(X, threshold, capacity=None, band_capacity=None):
    """Keys i*N + j (unordered, int64 GPU tensor) of every i < j with cosine(X_i, X_j) > threshold.
    X: (N, F) float64 GPU tensor.  Reruns once with exact buffer sizes if a capacity was short."""
    _req(X, torch.float64, None, "X")
    if X.dim() != 2:
        raise L.IddgcnError("X must be (N, F)")
    N, F = X.shape
    dev = X.device
    ws = _workspace(L.lib().iddgcn_similarity_workspace(N, F), dev)
    cap = int(capacity) if capacity is not None else max(1 << 16, 64 * N)
    bcap = int(band_capacity) if band_capacity is not None else max(1 << 14, 4 * N)
    counts = torch.empty(2, dtype=_I64, device=dev)
    for _ in range(2):
        keys = torch.empty(max(cap, 1), dtype=_I64, device=dev)
        band = torch.empty(max(bcap, 1), dtype=_I64, device=dev)
        L.check(L.lib().iddgcn_similarity_pairs(_stream(), N, F, _ptr(X), float(threshold), _ptr(keys), cap,
                                                _ptr(band), bcap, _ptr(counts), _ptr(ws), ws.numel()),
                "similarity_pairs")
        n_acc, n_band = (int(v) for v in counts.cpu())
        if n_acc <= cap and n_band <= bcap:
            return keys[:n_acc]
        cap, bcap = max(cap, n_acc), max(bcap, n_band)
    raise L.IddgcnError("similarity_pairs: capacity retry failed")


def similarity_triples(sorted_keys, N, relation, start):
    _req(sorted_keys, _I64, None, "sorted_keys")
    n = sorted_keys.shape[0]
    out = torch.empty((n, 3), dtype=_I64, device=sorted_keys.device)
    L.check(L.lib().iddgcn_similarity_triples(_stream(), n, N, int(relation), int(start), _ptr(sorted_keys),
                                              _ptr(out)), "similarity_triples")
    return out


# -- negative sampling (include/iddgcn_sampling.h) -----------------------------------------------
def mt19937_words(seed, n, device):
    """The first n words of np.random.seed(seed)'s MT19937 stream (tempered uint32, as int32 bits)."""
    state = torch.empty(625, dtype=_I32, device=device)
    L.check(L.lib().iddgcn_mt19937_seed(_stream(), int(seed), _ptr(state)), "mt19937_seed")
    out = torch.empty(max(int(n), 1), dtype=_I32, device=device)
    L.check(L.lib().iddgcn_mt19937_generate(_stream(), _ptr(state), int(n), _ptr(out)), "mt19937_generate")
    return out[:int(n)]


def negative_samples(triples, num_entities, seed):
    """utils1.generate_negative_samples_np (utils1.py:646-655) on the GPU, bit-exact: triples (M, 3)
    int64 GPU tensor -> (M, 3) int64 negatives.  Host synchronisations: one per round of entity words
    (normally one)."""
    _req(triples, _I64, None, "triples")
    if triples.dim() != 2 or triples.shape[1] != 3:
        raise L.IddgcnError(f"triples must be (M, 3), got {tuple(triples.shape)}")
    N = int(num_entities)
    if not 1 <= N <= 2 ** 31 - 1:
        raise L.IddgcnError("num_entities must be in [1, 2^31)")
    if not 0 <= int(seed) <= 2 ** 32 - 1:
        raise L.IddgcnError("seed must be between 0 and 2**32 - 1 (np.random.seed)")
    lib, dev, M = L.lib(), triples.device, triples.shape[0]
    out = torch.empty(M, 3, dtype=_I64, device=dev)
    if M == 0:
        return out
    state = torch.empty(625, dtype=_I32, device=dev)
    L.check(lib.iddgcn_mt19937_seed(_stream(), int(seed), _ptr(state)), "mt19937_seed")
    cond = torch.empty(M, dtype=_I32, device=dev)
    L.check(lib.iddgcn_mt19937_generate(_stream(), _ptr(state), M, _ptr(cond)), "mt19937_generate")
    ent = None
    if N > 1:
        rng = N - 1
        accept = (rng + 1) / (int(lib.iddgcn_randint_mask(rng)) + 1)       # > 1/2
        words = torch.empty(0, dtype=_I32, device=dev)
        ent = torch.empty(M, dtype=_I32, device=dev)
        need = M
        while True:
            more = int(need / accept * 1.01) + 4096
            new = torch.empty(more, dtype=_I32, device=dev)
            L.check(lib.iddgcn_mt19937_generate(_stream(), _ptr(state), more, _ptr(new)), "mt19937_generate")
            words = torch.cat([words, new]) if words.numel() else new
            nc = int(lib.iddgcn_accept_chunks(words.numel()))
            counts = torch.empty(nc, dtype=_I32, device=dev)
            offs = torch.empty(nc + 1, dtype=_I64, device=dev)
            L.check(lib.iddgcn_masked_accept(_stream(), _ptr(words), words.numel(), rng, M, _ptr(counts), _ptr(offs),
                                             _ptr(ent)), "masked_accept")
            got = int(offs[nc].item())
            if got >= M:
                break
            need = M - got
    L.check(lib.iddgcn_assemble_negatives(_stream(), M, _ptr(triples), _ptr(cond), _ptr(ent), _ptr(out)),
            "assemble_negatives")
    return out


PLANE_INV = 2.0 ** -15


def planes_to_f32(t):
    """Decode a pre-split planes table (include/iddgcn.h, IDDGCN_PLANES_*): rows of D = 256 in an
    fp32-shaped (rows, 256) tensor, 8 column blocks of [hi f16[32] | lo f16[32]], x = (hi + lo) * 2^-15."""
    h = t.contiguous().view(torch.float16).view(t.shape[0], t.shape[1] // 32, 2, 32)
    return ((h[:, :, 0].float() + h[:, :, 1].float()) * PLANE_INV).reshape(t.shape[0], t.shape[1])


def f32_to_planes(x):
    """The planes encoding of values in [0, 1] (round-to-nearest-even fp16 casts), as the producers write it."""
    xs = x.float() * 2.0 ** 15
    hi = xs.half()
    lo = (xs - hi.float()).half()
    rows = x.shape[0]
    return torch.stack([hi.view(rows, -1, 32), lo.view(rows, -1, 32)], 2).reshape(rows, -1).contiguous().view(torch.float32)
