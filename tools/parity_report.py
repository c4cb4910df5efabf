"""Measured parity numbers behind the GPU tests' bars, as one JSON file.

For every check: the HIP path's max abs error vs the float64 oracle, the fp32 oracle's own drift on the
same inputs (the reference computes in fp32), and the bar the test asserts.  Logits use the per-edge bar of
tests/parity.py (logit_report: also max |s - s32|, the distance to the fp32 oracle, the stand-in for TF's
fp32 output).  For the eval folds the per-layer outputs of every scored edge are compared too, so an excess
in the logits can be traced to the layer it enters.
usage (GPU box, repo root): python tools/parity_report.py > profiles/<round>/parity_report.json
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from iddgcn_amd import get_IDDGCN_Model  # noqa: E402
from iddgcn_amd.engine import Engine, FlatParams  # noqa: E402
from iddgcn_amd.graph import get_adj_mats  # noqa: E402
from iddgcn_amd.utils import synthetic_graph  # noqa: E402
from oracle.ref_model import forward_detail, init_params  # noqa: E402
from oracle.ref_utils import get_adj_coo as _coo  # noqa: E402,F811
from oracle.ref_utils import get_adj_coo  # noqa: E402
from parity import logit_report  # noqa: E402

G = os.path.join(ROOT, "tests", "golden")
load = lambda n: dict(np.load(os.path.join(G, n)))  # noqa: E731


def rec(err, drift, bar):
    return {"max_abs_err": float(err), "fp32_oracle_drift": float(drift), "bar": float(bar), "ok": bool(err <= bar)}


def main():
    dev = torch.device("cuda", 0)
    out = {"eval_logits": {}, "eval_probs": {}}
    for k in range(5):
        d, ev = load(f"fold{k}_data.npz"), load(f"fold{k}_eval.npz")
        model = get_IDDGCN_Model(845, 4, 64, 64, 1, None, 0, k)
        model.load_weights(os.path.join(G, f"weights_fold{k}.npz"))
        adj = get_adj_mats(np.concatenate([d["X_train"], d["X_test"]]), 845, 4)
        Xt = np.concatenate([d["X_test"], d["neg_X_test"]])[None]
        x = [np.arange(845)[None], Xt[:, :, 0], Xt[:, :, 1], Xt[:, :, 2], adj]
        s = model.predict_logits(x)[0].astype(np.float64)
        p = model.predict(x)[0].astype(np.float64)
        out["eval_logits"][f"fold{k}"] = logit_report(s, ev["logits"], ev["logits32"])
        out["eval_logits"][f"fold{k}"]["max_abs_logit"] = float(np.abs(ev["logits"]).max())
        out["eval_probs"][f"fold{k}"] = rec(np.abs(p - ev["probs"]).max(), np.abs(ev["probs32"] - ev["probs"]).max(),
                                            1e-4)
        # per-layer localisation on every eval edge: the engine's x_h^l, x_t^l vs the oracle in fp64 / fp32
        wk = load(f"weights_fold{k}.npz")
        tri = Xt[0].astype(np.int64)
        coo = _coo(np.concatenate([d["X_train"], d["X_test"]]), 845, 4)
        _, s64, l64 = forward_detail(wk, tri, coo, 845, dtype=torch.float64)
        _, s32, l32 = forward_detail(wk, tri, coo, 845, dtype=torch.float32)
        eng = Engine(845, 4, 64, dev)
        Pk = FlatParams(845, 4, 64, dev)
        Pk.load(wk)
        ed = eng.edges(tri)
        _, s_e = eng.predict(Pk, eng.adjacency(adj), ed, logits=True)
        loc = {"logits_engine": logit_report(s_e.cpu().numpy(), s64, s32)}
        for l, (xh, xt) in enumerate(eng.layer_outputs(ed), 1):
            for side, ours in ((0, xh), (1, xt)):
                o = ours.cpu().numpy().astype(np.float64)
                ref, r32 = np.asarray(l64[l - 1][side], np.float64), np.asarray(l32[l - 1][side], np.float64)
                loc[f"layer{l}_{'head' if side == 0 else 'tail'}"] = {
                    "max_err_vs_fp64": float(np.abs(o - ref).max()),
                    "max_err_vs_fp32_oracle": float(np.abs(o - r32).max()),
                    "max_fp32_drift": float(np.abs(r32 - ref).max())}
        out.setdefault("eval_layers", {})[f"fold{k}"] = loc
    g, d, w = load("fold0_step.npz"), load("fold0_data.npz"), load("weights_fold0.npz")
    eng = Engine(845, 4, 64, dev)
    P = FlatParams(845, 4, 64, dev)
    P.load(w)
    ed = eng.edges(np.concatenate([d["X_train"], d["X_train_neg"]]))
    _, s = eng.predict(P, eng.adjacency(get_adj_mats(d["X_train"], 845, 4)), ed, logits=True)
    out["fold0_step_logits"] = logit_report(s.cpu().numpy(), g["logits"], g["logits32"])
    out["fold0_layers_first256"] = {}
    for l, (xh, xt) in enumerate(eng.layer_outputs(ed, rows=np.arange(256)), 1):
        for side, ours in (("head", xh), ("tail", xt)):
            ref, r32 = g[f"layer{l}_{side}"], g[f"layer{l}_{side}32"]
            dr = np.abs(r32 - ref).max()
            out["fold0_layers_first256"][f"layer{l}_{side}"] = rec(np.abs(ours.cpu().numpy() - ref).max(), dr,
                                                                   max(1e-4, 2 * dr))
    # config 3 at full size, 10k-edge sample, every GEMM mode, mild and reference init
    N, R, M, D = 100_000, 2, 2_000_000, 256
    pos, neg = synthetic_graph(N, R, M, seed=0)
    tri = np.concatenate([pos, neg])
    eng = Engine(N, R, D, dev)
    adj = get_adj_mats(pos, N, R, device=dev)
    ed = eng.edges(tri)
    sample = np.sort(np.random.default_rng(0).choice(len(tri), 10_000, replace=False))
    coo = get_adj_coo(pos, N, R)
    from test_gpu_config3 import mild_params
    out["config3_sample10k"] = {}
    for init in ("mild", "reference"):
        params = mild_params() if init == "mild" else init_params(N, R, D, seed=89)
        p64, s64, l64 = forward_detail(params, tri[sample], coo, N, dtype=torch.float64)
        p32, s32, l32 = forward_detail(params, tri[sample], coo, N, dtype=torch.float32)
        P = FlatParams(N, R, D, dev)
        P.load(params)
        for gemm in ("split", "exact", "bf16x3"):
            eng.gemm = gemm
            p, s = eng.predict(P, adj, ed, logits=True)
            lay = eng.layer_outputs(ed, rows=sample)
            key = f"{init}/{gemm}"
            out["config3_sample10k"][key] = {
                "logits": logit_report(s.cpu().numpy()[sample], s64, s32),
                "probs": rec(np.abs(p.cpu().numpy()[sample] - p64).max(), np.abs(p32 - p64).max(), 1e-4),
                "layer3_tail": rec(np.abs(lay[2][1].cpu().numpy() - l64[2][1]).max(), np.abs(l32[2][1] - l64[2][1]).max(),
                                   max(1e-4, 2 * np.abs(l32[2][1] - l64[2][1]).max())),
                "max_abs_logit": float(np.abs(s64).max()),
            }
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
