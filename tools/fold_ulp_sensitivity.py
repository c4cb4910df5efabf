"""How far does a fold's 5000-epoch training move when its START moves by one fp32 ulp?

tools/fold_order_sensitivity.py re-orders a few of our own sums (the D = 64 projections / row GEMMs, the negatives'
order): a perturbation of a few ulps in a handful of ops per step.  The reference's TF-CPU arithmetic differs from
ours in every op of every step (per-edge GEMMs instead of node-level ones, TF's own reduction orders), so its
trajectory is perturbed from the first step on by more than those re-orderings.  This tool perturbs the replayed TF
2.7 start itself: every initial weight moved one ulp up or down (np.nextafter, random direction per element, seeds
1..S), then the reference's recipe (tests/test_gpu_training.py) for 5000 epochs.  Per fold it records the spread of
the runs (max rel. parameter distance, per parameter max |w - w'| / max |w'|, between every perturbed run and the
unperturbed one), each run's distance to the bundled trained weights, and the eval AUC.

usage: python tools/fold_ulp_sensitivity.py [--folds 0,1,2,3,4] [--seeds 3] [--epochs 5000] [--out FILE]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from sklearn.metrics import roc_auc_score  # noqa: E402

from iddgcn_amd import Adam, BinaryCrossentropy, get_IDDGCN_Model  # noqa: E402
from iddgcn_amd.graph import get_adj_mats  # noqa: E402

N_ENT, N_REL, DIM = 845, 4, 64


def rel(a, b):
    return {k: float(np.abs(a[k] - b[k]).max() / max(np.abs(b[k]).max(), 1e-30)) for k in b}


def run(fold, d, epochs, seed):
    kw = dict(tf_models_before=1, tf_extra_op_seeds=1) if fold == 3 else {}
    model = get_IDDGCN_Model(N_ENT, N_REL, DIM, DIM, 89, None, 0, fold, init="tf27", **kw)
    if seed:
        rng = np.random.RandomState(seed)
        w = model._named()
        for k, v in w.items():
            if k.startswith("relw"):            # never trained (IDDGCN.py:39-44): left as drawn
                continue
            up = rng.randint(0, 2, v.shape).astype(bool)
            w[k] = np.where(up, np.nextafter(v, np.float32(np.inf)), np.nextafter(v, np.float32(-np.inf))).astype(np.float32)
        model._set_named(w)
    model.neg_triples = d["X_train_neg"][None]
    model.compile(loss=BinaryCrossentropy(), optimizer=Adam(learning_rate=0.001))
    X = d["X_train"][None]
    model.fit(x=[np.arange(N_ENT)[None], X[:, :, 0], X[:, :, 1], X[:, :, 2], get_adj_mats(d["X_train"], N_ENT, N_REL)],
              y=np.ones((1, X.shape[1])), epochs=epochs, batch_size=100, verbose=0)
    adj = get_adj_mats(np.concatenate([d["X_train"], d["X_test"]]), N_ENT, N_REL)
    Xt = np.concatenate([d["X_test"], d["neg_X_test"]])[None]
    y = np.concatenate([np.ones(len(d["X_test"])), np.zeros(len(d["neg_X_test"]))])
    p = model.predict(x=[np.arange(N_ENT)[None], Xt[:, :, 0], Xt[:, :, 1], Xt[:, :, 2], adj])[0]
    model._sync_to_host()
    return {k: v.copy() for k, v in model._named().items()}, float(roc_auc_score(y, p))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--folds", default="0,1,2,3,4")
    ap.add_argument("--seeds", type=int, default=3)
    ap.add_argument("--epochs", type=int, default=5000)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    out = {}
    for fold in map(int, a.folds.split(",")):
        d = dict(np.load(os.path.join(ROOT, "tests", "golden", f"fold{fold}_data.npz")))
        ref = dict(np.load(os.path.join(ROOT, "tests", "golden", f"weights_fold{fold}.npz")))
        runs = {s: run(fold, d, a.epochs, s) for s in range(a.seeds + 1)}
        w0 = runs[0][0]
        rec = {"runs": {}}
        for s, (w, auc) in runs.items():
            vb, v0 = rel(w, ref), rel(w, w0)
            rec["runs"][s] = {"auc": auc, "vs_bundled_max": max(vb.values()), "vs_bundled_argmax": max(vb, key=vb.get),
                              "vs_unperturbed_max": max(v0.values()), "vs_unperturbed_argmax": max(v0, key=v0.get),
                              "vs_bundled": vb, "vs_unperturbed": v0}
        rec["spread_max"] = max(r["vs_unperturbed_max"] for r in rec["runs"].values())
        out[fold] = rec
        print(json.dumps({"fold": fold, "spread_max": rec["spread_max"],
                          "runs": {s: {k: r[k] for k in ("auc", "vs_bundled_max", "vs_bundled_argmax", "vs_unperturbed_max")}
                                   for s, r in rec["runs"].items()}}), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
