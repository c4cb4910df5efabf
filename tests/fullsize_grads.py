"""Full-size backward parity against the oracle (IDDGCN.py:146-174: tape.gradient of the scaled Keras BCE).

The oracle (oracle/ref_model.py: torch autograd of the reference formulation) cannot run a 40M-edge step, but a
step's gradients are sums over scored edges, so a SAMPLE of scored edges is an exact smaller problem:

  * the engine runs ``loss_and_grads`` on the sampled scored edges with the workload's FULL device adjacency and
    full node tables: million-row AE / P / dP / dAE tables (R·N·D up to 2^31 elements at config 5), the
    transposed SpMM over every adjacency entry (20M / 40M nnz), head / tail segment pointers over all N nodes;
  * the oracle runs the reference formulation on the same scored edges with the adjacency rows the forward
    gathers (A_r·E is only read at the sampled heads and tails, IDDGCN.py:71-72), relabelled monotonically onto
    the entities those rows touch (order-preserving, so get_adj_coo's sorted order and every op order are
    unchanged), with the loss scale ×1/num_entities of the FULL graph (:168).  Its dE is scattered back to N rows:
    every other row of the engine's dE must be exactly zero.

The sample is random scored edges plus every scored edge of a few tails and heads drawn by degree (complete tail /
head segments at the workload's natural lengths, ~100-200 edges at the drug nodes), so the segmented reductions see
long segments as well as the scattered single edges.
"""
import json
import os

import numpy as np
import torch

from iddgcn_amd.engine import FlatParams
from oracle.ref_model import train_step_grads
from oracle.ref_utils import get_adj_coo


def grad_sample(tri, n_random=6000, n_tail=24, n_head=24, seed=0):
    """Sorted indices into ``tri``: ``n_random`` random scored edges plus every scored edge whose tail is one of
    ``n_tail`` entities, or whose head is one of ``n_head`` entities, drawn as endpoints of random scored edges
    (i.e. by degree)."""
    rng = np.random.default_rng(seed)
    pick = rng.choice(len(tri), n_random, replace=False)
    tails = np.unique(tri[rng.choice(len(tri), n_tail, replace=False), 2])
    heads = np.unique(tri[rng.choice(len(tri), n_head, replace=False), 0])
    seg = np.flatnonzero(np.isin(tri[:, 2], tails) | np.isin(tri[:, 0], heads))
    return np.union1d(pick, seg)


def local_oracle(params, pos, tri_s, lab_s, N, R, dtype):
    """train_step_grads on the sampled scored edges, relabelled onto the entities the forward touches.
    Returns (mean loss, probabilities in tri_s order, grads with E scattered back to N rows, those entities)."""
    rows = np.unique(np.concatenate([tri_s[:, 0], tri_s[:, 2]]))
    sub = pos[np.isin(pos[:, 0], rows)]
    for r in range(R):
        assert (sub[:, 1] == r).any(), "a relation without entries in the sample's rows (placeholder semantics)"
    ents = np.unique(np.concatenate([rows, sub[:, 2]]))
    loc = lambda t: np.stack([np.searchsorted(ents, t[:, 0]), t[:, 1], np.searchsorted(ents, t[:, 2])], 1)  # noqa
    coo = get_adj_coo(loc(sub), len(ents), R)
    p_l = dict(params)
    p_l["E"] = np.ascontiguousarray(params["E"][ents])
    is_pos = lab_s > 0.5
    assert is_pos[:is_pos.sum()].all(), "sample must list positives first (the oracle's pos ++ neg order)"
    tl = loc(tri_s)
    loss, scores, g = train_step_grads(p_l, tl[is_pos], tl[~is_pos], coo, len(ents), dtype=dtype, scale_entities=N)
    gE = np.zeros((N, params["E"].shape[1]), dtype=g["E"].dtype)
    gE[ents] = g["E"]
    g["E"] = gE
    return loss, scores, g, ents


def engine_grads(eng, P, adj, tri_s, lab_s, gemm, cuda):
    """The engine's loss_and_grads on the sampled scored edges with the FULL device adjacency.  ``gemm``: the
    engine's GEMM mode, optionally "/bf16" for bf16 edge-GEMM operands (Engine.edge_mfma, bf16 edge tables)."""
    mode, _, em = gemm.partition("/")
    eng.gemm = mode
    eng.edge_mfma = em or "hilo"
    ed = eng.edges(tri_s, lab_s)
    G = FlatParams(eng.N, eng.R, eng.D, cuda)
    loss_sum, p = eng.loss_and_grads(P, G, adj, ed)
    out = (float(loss_sum.item()) / len(tri_s), p.cpu().numpy(), G.to_numpy())
    del G, ed
    eng.edge_mfma = "hilo"
    eng.release()
    return out


def check_sampled_grads(eng, adj, params, pos, tri_s, lab_s, gemms, cuda, saturating, what, bar=2e-4, loss_bar=1e-5,
                        p_bar=1e-5):
    """Every gradient of the sampled step, per GEMM mode, against the float64 oracle.

    Non-saturating init (``saturating=False``): loss ``loss_bar`` rel (1e-5), probabilities ``p_bar`` (1e-5), every
    gradient within ``bar`` (2e-4) of its max |g|.  Reference init (saturating sigmoids): each quantity within max(bar, 2x the fp32 oracle's own
    distance from float64), the bar the fold-0 trained-weights step uses (tests/test_gpu_model.py)."""
    N, R = eng.N, eng.R
    l64, s64, g64, ents = local_oracle(params, pos, tri_s, lab_s, N, R, torch.float64)
    if saturating:
        l32, s32, g32, _ = local_oracle(params, pos, tri_s, lab_s, N, R, torch.float32)
    outside = np.ones(N, bool)
    outside[ents] = False
    assert all(np.all(np.isfinite(v)) for v in g64.values())
    P = FlatParams(N, R, eng.D, cuda)
    P.load(params)
    report = {}
    for gemm in gemms:
        loss, p, g = engine_grads(eng, P, adj, tri_s, lab_s, gemm, cuda)
        lerr = abs(loss - l64) / abs(l64)
        perr = np.abs(p.astype(np.float64) - s64).max()
        lbar = max(loss_bar, 2 * abs(l32 - l64) / abs(l64)) if saturating else loss_bar
        pbar = max(1e-4, 2 * np.abs(s32 - s64).max()) if saturating else p_bar
        assert lerr <= lbar, f"{what} {gemm}: loss rel err {lerr:.2e} > {lbar:.2e}"
        assert perr <= pbar, f"{what} {gemm}: probabilities {perr:.2e} > {pbar:.2e}"
        rep = {}
        for k, ref in g64.items():
            ours = g[k].astype(np.float64)
            assert np.all(np.isfinite(ours)), (what, gemm, k)
            scale = np.abs(ref).max()
            err = np.abs(ours - ref).max() / scale
            kb = max(bar, 2 * np.abs(g32[k].astype(np.float64) - ref).max() / scale) if saturating else bar
            rep[k] = (err, kb)
            assert err <= kb, f"{what} {gemm}: grad {k} max err {err:.2e} of max|g| > bar {kb:.2e}"
        # rows of dE outside the sampled edges' reach (no path from the loss: not a sampled head / tail, not in
        # their adjacency rows) are exactly zero
        assert not np.any(g["E"][outside]), f"{what} {gemm}: nonzero dE rows outside the sample's entities"
        report[gemm] = {"loss_rel_err": lerr, "loss_bar": lbar, "p_err": float(perr), "p_bar": pbar,
                        "grads": {k: {"err_of_max": float(e), "bar": float(b)} for k, (e, b) in rep.items()}}
    del P
    log = os.environ.get("IDDGCN_PARITY_LOG")    # e.g. gpurun_out/<tag>/fullsize_grads.jsonl: the measured record
    if log:
        with open(log, "a") as f:
            f.write(json.dumps({"what": what, "n_scored": int(len(tri_s)), "n_entities_reached": int(len(ents)),
                                "modes": report}) + "\n")
    return report
