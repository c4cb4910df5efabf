"""Train IDDGCN from scratch on the bundled 5-fold split and evaluate it as IDDGCN_eval.py does.

This is the reference's training driver (IDDGCN.py:287-412: get_IDDGCN_Model, compile with
BinaryCrossentropy + Adam(1e-3), full-batch fit for 5000 epochs on the fold's X_train and its .npy
negatives) followed by its evaluation (IDDGCN_eval.py:35-122: adjacency from X_train plus the test
positives, predict on test positives + negatives, ROC-AUC / AUPR / accuracy at 0.5), on the HIP path
through the Keras-shaped API.  Fold data are the reference's bundled files (tests/golden/fold*_data.npz).
With the default init "tf27" and seed 89 each fold starts from the reference's own initial weights (TF 2.7's
draws replayed, iddgcn_amd/tf_random.py; fold 3 as the second model of its process, as its bundled
relation_weights show), so a fold's AUC is compared with the AUC of the weights the reference trained from that
same start; other seeds / "independent" give the spread.

usage: python tools/train_folds.py [--folds 0,1,2,3,4] [--seeds 89,1,2] [--epochs 5000] [--init tf27]
                                  [--out FILE]
"""
import argparse
import json
import os
import statistics
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from sklearn.metrics import auc, precision_recall_curve, roc_auc_score  # noqa: E402

from iddgcn_amd import Adam, BinaryCrossentropy, get_IDDGCN_Model  # noqa: E402
from iddgcn_amd.graph import get_adj_mats  # noqa: E402

N_ENT, N_REL, DIM = 845, 4, 64
# ROC-AUC of the reference's bundled trained weights under the oracle's eval restatement (not
# published numbers: the reference publishes none)
REFERENCE_WEIGHTS_AUC = {0: 0.9072, 1: 0.8841, 2: 0.8832, 3: 0.9148, 4: 0.9068}


def run(fold, seed, epochs, init="tf27"):
    d = np.load(os.path.join(ROOT, "tests", "golden", f"fold{fold}_data.npz"))
    # the bundled fold-3 weights were trained as the second model of a process (tests/test_tf_random.py)
    kw = dict(tf_models_before=1, tf_extra_op_seeds=1) if (init == "tf27" and fold == 3 and seed == 89) else {}
    model = get_IDDGCN_Model(N_ENT, N_REL, DIM, DIM, seed, None, 0, fold, init=init, **kw)
    model.neg_triples = d["X_train_neg"][None]
    model.compile(loss=BinaryCrossentropy(), optimizer=Adam(learning_rate=0.001))
    X = d["X_train"][None]
    adj = get_adj_mats(d["X_train"], N_ENT, N_REL)
    t0 = time.perf_counter()
    hist = model.fit(x=[np.arange(N_ENT)[None], X[:, :, 0], X[:, :, 1], X[:, :, 2], adj],
                     y=np.ones((1, X.shape[1])), epochs=epochs, batch_size=100, verbose=0)
    train_s = time.perf_counter() - t0
    # IDDGCN_eval.py: the test positives are part of the message-passing graph
    adj_eval = get_adj_mats(np.concatenate([d["X_train"], d["X_test"]]), N_ENT, N_REL)
    Xt = np.concatenate([d["X_test"], d["neg_X_test"]])[None]
    y = np.concatenate([np.ones(len(d["X_test"])), np.zeros(len(d["neg_X_test"]))])
    p = model.predict(x=[np.arange(N_ENT)[None], Xt[:, :, 0], Xt[:, :, 1], Xt[:, :, 2], adj_eval])[0]
    prec, reca, _ = precision_recall_curve(y, p)
    # the reference trained its bundled weights from this same start (tf27, seed 89) with the same deterministic
    # full-batch loop: how far the trained weights land from them, per parameter (max |w - w_ref| / max |w_ref|)
    wdiff = None
    if init == "tf27" and seed == 89:
        model._sync_to_host()
        ref = np.load(os.path.join(ROOT, "tests", "golden", f"weights_fold{fold}.npz"))
        mine = model._named()
        wdiff = {k: float(np.abs(mine[k] - ref[k]).max() / max(np.abs(ref[k]).max(), 1e-30)) for k in ref.files}
        pr = model.predict(x=[np.arange(N_ENT)[None], Xt[:, :, 0], Xt[:, :, 1], Xt[:, :, 2], adj_eval])[0]
        assert np.array_equal(pr, p)
    return {"fold": fold, "seed": seed, "init": init, "epochs": epochs, "train_s": train_s,
            "trained_vs_bundled_weights_rel": wdiff,
            "ms_per_epoch": train_s / epochs * 1e3, "final_loss": hist.history["loss"][-1],
            "roc_auc": float(roc_auc_score(y, p)), "aupr": float(auc(reca, prec)),
            "accuracy": float(((p > 0.5) == (y > 0.5)).mean()), "reference_weights_auc_restated": REFERENCE_WEIGHTS_AUC[fold]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--folds", default="0,1,2,3,4")
    ap.add_argument("--seeds", default="89,1,2")
    ap.add_argument("--epochs", type=int, default=5000)
    ap.add_argument("--out", default=None)
    ap.add_argument("--init", default="tf27", choices=["tf27", "independent"],
                    help="weight-initialisation scheme (iddgcn_amd.model.INIT_SCHEMES)")
    a = ap.parse_args()
    runs = []
    for fold in map(int, a.folds.split(",")):
        for seed in map(int, a.seeds.split(",")):
            r = run(fold, seed, a.epochs, a.init)
            runs.append(r)
            print(json.dumps(r), flush=True)
    summary = {}
    for fold in sorted({r["fold"] for r in runs}):
        aucs = [r["roc_auc"] for r in runs if r["fold"] == fold]
        summary[fold] = {"roc_auc_mean": statistics.mean(aucs),
                         "roc_auc_sd": statistics.stdev(aucs) if len(aucs) > 1 else 0.0,
                         "reference_weights_auc_restated": REFERENCE_WEIGHTS_AUC[fold], "n_seeds": len(aucs)}
    out = {"runs": runs, "summary": summary}
    print(json.dumps(summary), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
