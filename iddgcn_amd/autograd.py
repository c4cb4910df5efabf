"""Differentiable layer-level calls: torch.autograd.Functions over the HIP kernels.

The reference's ``IDDGCN_Layer`` and ``DistMult`` (prediction/IDDGCN.py:16-109) are Keras layers, so a
caller can build other models from them and differentiate through them with ``tf.GradientTape``.
``IDDGCNLayerFunction`` / ``DistMultFunction`` give the same on torch tensors; ``model.IDDGCN_Layer`` /
``model.DistMult`` route through them.  The full training step does not use these (engine.Engine runs the
node-level formulation with its own backward); they are the per-call form, edge by edge as the
reference's layer computes:

forward (IDDGCN.py:60-79):   AE_r = A_r E;  P_r = AE_r K_r;  w = sigmoid(softmax(x_h Wa + ba));
                             o_h = sigmoid(x_h S + sum_r w_r P_r[h]);  o_t = sigmoid(x_t S + sum_r w_r P_r[t])
backward:  g_h = do_h o_h (1 - o_h), g_t likewise;  dS = x_h^T g_h + x_t^T g_t;
           dw_r = <g_h, P_r[h]> + <g_t, P_r[t]>  ->  dz (softmax-sigmoid)  ->  dWa = x_h^T dz, dba = sum dz;
           dx_h = g_h S^T + dz Wa^T;  dx_t = g_t S^T;
           dP_r[n] = sum_{h_e = n} w_r g_h[e] + sum_{t_e = n} w_r g_t[e]  (segmented, deterministic);
           dK_r = AE_r^T dP_r;  dE = sum_r A_r^T (dP_r K_r^T).
Every GEMM, SpMM and segmented reduction is a libiddgcn_hip kernel; torch supplies the elementwise glue
and the index sorts of the edge batch.
"""
import torch

from . import _lib as L
from . import ops


def _segments(idx, n):
    """Stable order of the edges by node and the CSR-style segment pointers (n + 1)."""
    order = torch.sort(idx.long(), stable=True).indices
    ptr = torch.searchsorted(idx.long()[order], torch.arange(n + 1, device=idx.device)).to(torch.int32)
    return order, ptr.contiguous()


class IDDGCNLayerFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, E, head_e, tail_e, K, S, Wa, ba, head_idx, tail_idx, dadj):
        N, D = E.shape
        R = K.shape[0]
        B = head_e.shape[0]
        dev = E.device
        E, head_e, tail_e = E.contiguous(), head_e.contiguous(), tail_e.contiguous()
        K, S, Wa, ba = K.contiguous(), S.contiguous(), Wa.contiguous(), ba.contiguous()
        AE = torch.empty(R, N, D, device=dev)
        ops.spmm_csr(dadj.fwd_ptr, dadj.fwd_col, dadj.fwd_val, E, AE, R, N)
        P = torch.empty(R, N, D, device=dev)
        ops.rowgemm_batched([(AE[r], K[r], P[r], {}) for r in range(R)])
        Ssm, W = torch.empty(B, R, device=dev), torch.empty(B, R, device=dev)
        ops.alpha_fwd(head_e, Wa, ba, Ssm, W)
        ho, to = torch.empty(B, D, device=dev), torch.empty(B, D, device=dev)
        ops.rowgemm(head_e, S, ho, coef=W, V=P, v_idx=head_idx, v_rel_stride=N * D, act=L.ACT_SIGMOID)
        ops.rowgemm(tail_e, S, to, coef=W, V=P, v_idx=tail_idx, v_rel_stride=N * D, act=L.ACT_SIGMOID)
        ctx.save_for_backward(head_e, tail_e, K, S, Wa, AE, P, Ssm, W, ho, to, head_idx, tail_idx)
        ctx.dadj = dadj
        return ho, to

    @staticmethod
    def backward(ctx, dho, dto):
        head_e, tail_e, K, S, Wa, AE, P, Ssm, W, ho, to, head_idx, tail_idx = ctx.saved_tensors
        dadj = ctx.dadj
        R, N, D = P.shape
        B = head_e.shape[0]
        dev = P.device
        dho = torch.zeros_like(ho) if dho is None else dho.contiguous()
        dto = torch.zeros_like(to) if dto is None else dto.contiguous()
        gh = (dho * ho * (1 - ho)).contiguous()
        gt = (dto * to * (1 - to)).contiguous()
        slab = torch.empty(max(ops.tn_blocks(B, D), ops.tn_blocks(N, D)) * D * D, device=dev)
        dS = torch.empty(D, D, device=dev)
        ops.gemm_tn(head_e, gh, dS, slab)
        ops.gemm_tn(tail_e, gt, dS, slab, accumulate=True)
        # per-side segmented reductions: dP_r (w_r-weighted sums of the rows per node) and dw_r
        dP = torch.zeros(R, N, D, device=dev)
        dw = torch.zeros(B, R, device=dev)
        for idx, g in ((head_idx, gh), (tail_idx, gt)):
            order, ptr = _segments(idx, N)
            dP_s, dw_s = torch.empty(R, N, D, device=dev), torch.empty(B, R, device=dev)
            ops.tail_seg_reduce(ptr, None, W[order].contiguous(), g[order].contiguous(), P, dP_s, dw_s)
            dP += dP_s
            dw[order] += dw_s
        # softmax-sigmoid backward of w = sigmoid(softmax(z))
        ds = dw * W * (1 - W)
        dz = (Ssm * (ds - (ds * Ssm).sum(1, keepdim=True))).contiguous()
        dWa, dba = torch.empty_like(Wa), torch.empty(R, device=dev)
        narrow = torch.empty((ops.tn_narrow_blocks(B) + 1) * (D + 1) * R, device=dev)
        ops.gemm_tn_narrow(head_e, dz, dWa, dba, narrow)
        dhe, dte = torch.empty_like(head_e), torch.empty_like(tail_e)
        ops.rowgemm(gh, S, dhe, b_trans=True, coef=dz, V=Wa.t().contiguous(), v_rel_stride=D, v_row_stride=0)
        ops.rowgemm(gt, S, dte, b_trans=True)
        dK = torch.empty_like(K)
        for r in range(R):
            ops.gemm_tn(AE[r], dP[r], dK[r], slab)
        dAE = torch.empty(R, N, D, device=dev)
        ops.rowgemm_batched([(dP[r], K[r], dAE[r], dict(b_trans=True)) for r in range(R)])
        dE = torch.zeros(N, D, device=dev)
        ops.spmm_csr(dadj.bwd_ptr, dadj.bwd_col, dadj.bwd_val, dAE.view(R * N, D), dE.view(1, N, D), 1, N,
                     accumulate=True)
        return dE, dhe, dte, dK, dS, dWa, dba, None, None, None


class DistMultFunction(torch.autograd.Function):
    """p = sigmoid(sum_d h_d rel[r]_d t_d) (IDDGCN.py:103-109), forward on the DistMult kernel."""

    @staticmethod
    def forward(ctx, head_e, rel, tail_e, rel_idx):
        B = head_e.shape[0]
        dev = head_e.device
        head_e, tail_e, rel = head_e.contiguous(), tail_e.contiguous(), rel.contiguous()
        ident = torch.arange(B, device=dev, dtype=torch.int32)
        p = torch.empty(B, device=dev)
        ops.distmult_bce(head_e, ident, tail_e, rel_idx, rel, p_out=p)
        ctx.save_for_backward(head_e, rel, tail_e, rel_idx, p)
        return p

    @staticmethod
    def backward(ctx, dp):
        head_e, rel, tail_e, rel_idx, p = ctx.saved_tensors
        ds = (dp * p * (1 - p))[:, None]
        rho = rel[rel_idx.long()]
        onehot = torch.nn.functional.one_hot(rel_idx.long(), rel.shape[0]).to(ds.dtype)
        drel = onehot.t() @ (ds * head_e * tail_e)          # deterministic per-relation sums
        return ds * rho * tail_e, drel, ds * rho * head_e, None
