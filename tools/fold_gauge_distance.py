"""Fold distance to the bundled trained weights, with and without the softmax gauge of the attention weights.

alpha = softmax(h W_alpha + b_alpha) over the R relations (IDDGCN.py:66) does not change when the same vector is added
to every column of W_alpha and the same constant to every entry of b_alpha: per layer, D + 1 directions of the
parameters the loss cannot see.  The gradient has no component along them (each row of d alpha / d logits sums to
zero over r), but Keras Adam's per-element normalisation (m / (sqrt(v) + eps)) does not preserve that zero sum, so
where a run drifts along these directions depends on its whole gradient history, not on the model it computes.
This tool trains each fold 5000 epochs from the replayed TF 2.7 start (the recipe of tests/test_gpu_training.py)
and reports, per parameter, the max relative distance to the bundled weights (max |w - w_ref| / max |w_ref|) both raw
and after removing the gauge (W_alpha and b_alpha centred over relations, which leaves alpha unchanged), beside the
distance of what the model computes: max |p - p_ref| of the eval probabilities, the training loss, and the layer
attention alpha^l on every node.

usage: python tools/fold_gauge_distance.py [--folds 0,1,2,3,4] [--epochs 5000] [--out FILE]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from iddgcn_amd import Adam, BinaryCrossentropy, get_IDDGCN_Model  # noqa: E402
from iddgcn_amd.graph import get_adj_mats  # noqa: E402

N_ENT, N_REL, DIM = 845, 4, 64


def rel(a, b):
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


def centred(w):
    """W_alpha (D x R) and b_alpha (R,) with their mean over relations removed: the same softmax."""
    w = dict(w)
    for l in (1, 2, 3):
        w[f"Wa{l}"] = w[f"Wa{l}"] - w[f"Wa{l}"].mean(axis=1, keepdims=True)
        w[f"ba{l}"] = w[f"ba{l}"] - w[f"ba{l}"].mean()
    return w


def softmax(z):
    z = z - z.max(axis=1, keepdims=True)
    e = np.exp(z)
    return e / e.sum(axis=1, keepdims=True)


def eval_probs(model, d):
    adj = get_adj_mats(np.concatenate([d["X_train"], d["X_test"]]), N_ENT, N_REL)
    Xt = np.concatenate([d["X_test"], d["neg_X_test"]])[None]
    return model.predict(x=[np.arange(N_ENT)[None], Xt[:, :, 0], Xt[:, :, 1], Xt[:, :, 2], adj])[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--folds", default="0,1,2,3,4")
    ap.add_argument("--epochs", type=int, default=5000)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    out = {}
    for fold in map(int, a.folds.split(",")):
        d = dict(np.load(os.path.join(ROOT, "tests", "golden", f"fold{fold}_data.npz")))
        ref = dict(np.load(os.path.join(ROOT, "tests", "golden", f"weights_fold{fold}.npz")))
        kw = dict(tf_models_before=1, tf_extra_op_seeds=1) if fold == 3 else {}
        model = get_IDDGCN_Model(N_ENT, N_REL, DIM, DIM, 89, None, 0, fold, init="tf27", **kw)
        model.neg_triples = d["X_train_neg"][None]
        model.compile(loss=BinaryCrossentropy(), optimizer=Adam(learning_rate=0.001))
        X = d["X_train"][None]
        model.fit(x=[np.arange(N_ENT)[None], X[:, :, 0], X[:, :, 1], X[:, :, 2], get_adj_mats(d["X_train"], N_ENT, N_REL)],
                  y=np.ones((1, X.shape[1])), epochs=a.epochs, batch_size=100, verbose=0)
        model._sync_to_host()
        w = model._named()
        ref_model = get_IDDGCN_Model(N_ENT, N_REL, DIM, DIM, 89, None, 0, fold, init="tf27", **kw)
        ref_model.load_weights(os.path.join(ROOT, "tests", "golden", f"weights_fold{fold}.npz"))
        raw = {k: rel(w[k], ref[k]) for k in ref}
        wc, rc = centred(w), centred(ref)
        gauge_free = {k: rel(wc[k], rc[k]) for k in ref}
        # the gauge component itself: the relation-mean of W_alpha / b_alpha, ours vs the bundled file
        gauge = {f"Wa{l}_mean_over_r": (float(np.abs(w[f"Wa{l}"].mean(1)).max()), float(np.abs(ref[f"Wa{l}"].mean(1)).max()))
                 for l in (1, 2, 3)}
        p, pr = eval_probs(model, d), eval_probs(ref_model, d)
        rec = {"raw_max": max(raw.values()), "raw_argmax": max(raw, key=raw.get),
               "gauge_free_max": max(gauge_free.values()), "gauge_free_argmax": max(gauge_free, key=gauge_free.get),
               "raw": raw, "gauge_free": gauge_free, "gauge_component_max_abs": gauge,
               "eval_prob_max_abs_diff": float(np.abs(p - pr).max()),
               "eval_prob_mean_abs_diff": float(np.abs(p - pr).mean())}
        out[fold] = rec
        print(json.dumps({"fold": fold, **{k: rec[k] for k in ("raw_max", "raw_argmax", "gauge_free_max", "gauge_free_argmax",
                                                           "eval_prob_max_abs_diff", "eval_prob_mean_abs_diff")}}),
              flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
