"""Distance of a fold's trained weights to the reference's bundled trained weights along the training run (every
``--every`` epochs up to ``--epochs``), from the replayed TF 2.7 start (VERDICT r04 "explain fold 4": is the bundled
fold-4 file the end point of a 5000-epoch run from that start, or of another length / path?).

usage: python tools/fold_epoch_sweep.py [--folds 4,0] [--epochs 8000] [--every 100] [--out FILE]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--folds", default="4,0")
    ap.add_argument("--epochs", type=int, default=8000)
    ap.add_argument("--every", type=int, default=100)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    out = {}
    for fold in map(int, a.folds.split(",")):
        d = np.load(os.path.join(ROOT, "tests", "golden", f"fold{fold}_data.npz"))
        ref = dict(np.load(os.path.join(ROOT, "tests", "golden", f"weights_fold{fold}.npz")))
        kw = dict(tf_models_before=1, tf_extra_op_seeds=1) if fold == 3 else {}
        model = get_IDDGCN_Model(N_ENT, N_REL, DIM, DIM, 89, None, 0, fold, init="tf27", **kw)
        model.neg_triples = d["X_train_neg"][None]
        model.compile(loss=BinaryCrossentropy(), optimizer=Adam(learning_rate=0.001))
        X = d["X_train"][None]
        x = [np.arange(N_ENT)[None], X[:, :, 0], X[:, :, 1], X[:, :, 2], get_adj_mats(d["X_train"], N_ENT, N_REL)]
        rows, done = [], 0
        while done < a.epochs:
            h = model.fit(x=x, y=np.ones((1, X.shape[1])), epochs=a.every, batch_size=100, verbose=0)
            done += a.every
            model._sync_to_host()
            w = model._named()
            r = {k: float(np.abs(w[k] - ref[k]).max() / max(np.abs(ref[k]).max(), 1e-30)) for k in ref}
            rows.append({"epoch": done, "loss": h.history["loss"][-1], "max": max(r.values()),
                         "argmax": max(r, key=r.get), "E": r["E"], "Wa3": r["Wa3"]})
        best = min(rows, key=lambda z: z["max"])
        out[fold] = {"rows": rows, "closest": best}
        print(json.dumps({"fold": fold, "closest": best, "at_5000": next(z for z in rows if z["epoch"] == 5000)}),
              flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
