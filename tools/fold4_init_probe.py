"""Fold 4's bundled trained weights sit 25-27% (max rel. parameter distance) from every run of ours from the replayed
TF 2.7 start, at every epoch up to 9000 (tools/fold_epoch_sweep.py), while five re-orderings of our own arithmetic
stay within 2% of each other (tools/fold_order_sensitivity.py): a difference in what the reference started from or
trained on, not rounding.  The replay pins the fold's relation_weights (op seeds #0, #2, #4: a fresh op-seed counter)
and its untouched entity rows (the seeded uniform kernel from counter 0); the seeded NORMAL draws (relation / self
kernels, DistMult's relation embedding) are trained and so unpinned.  This probe starts fold 4 from inits whose
seeded normal kernel had already run m models' worth of draws (m = 0..4: what a process that built m models before
and then re-set the seed, which restarts the op-seed counter but not eager mode's cached seeded kernels, would draw),
trains 5000 epochs and reports each run's distance to the bundled weights.

usage: python tools/fold4_init_probe.py [--fold 4] [--m 0,1,2,3,4] [--out FILE]
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
from iddgcn_amd.tf_random import TFRandom, draw_model  # noqa: E402

N_ENT, N_REL, DIM = 845, 4, 64


def init_with_normal_offset(m, seed=89):
    tf = TFRandom(seed)
    for _ in range(m):
        for _l in (1, 2, 3):
            tf.normal((N_REL, DIM, DIM), 0.0, 1.0, seed=seed)
            tf.normal((DIM, DIM), 0.0, 1.0, seed=seed)
        tf.normal((N_REL, DIM), 0.0, 1.0, seed=seed)
    return draw_model(tf, N_ENT, N_REL, DIM, seed)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fold", type=int, default=4)
    ap.add_argument("--m", default="0,1,2,3,4")
    ap.add_argument("--epochs", type=int, default=5000)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    d = np.load(os.path.join(ROOT, "tests", "golden", f"fold{a.fold}_data.npz"))
    ref = dict(np.load(os.path.join(ROOT, "tests", "golden", f"weights_fold{a.fold}.npz")))
    X = d["X_train"][None]
    x = [np.arange(N_ENT)[None], X[:, :, 0], X[:, :, 1], X[:, :, 2], get_adj_mats(d["X_train"], N_ENT, N_REL)]
    out = []
    for m in map(int, a.m.split(",")):
        init = init_with_normal_offset(m)
        assert all(np.array_equal(init[f"relw{l}"], ref[f"relw{l}"]) for l in (1, 2, 3))
        model = get_IDDGCN_Model(N_ENT, N_REL, DIM, DIM, 89, None, 0, a.fold, init="tf27")
        model._set_named(init)
        model._invalidate()
        model.neg_triples = d["X_train_neg"][None]
        model.compile(loss=BinaryCrossentropy(), optimizer=Adam(learning_rate=0.001))
        model.fit(x=x, y=np.ones((1, X.shape[1])), epochs=a.epochs, batch_size=100, verbose=0)
        model._sync_to_host()
        w = model._named()
        r = {k: float(np.abs(w[k] - ref[k]).max() / max(np.abs(ref[k]).max(), 1e-30)) for k in ref}
        row = {"m": m, "max": max(r.values()), "argmax": max(r, key=r.get), "per_param": r}
        out.append(row)
        print(json.dumps({k: v for k, v in row.items() if k != "per_param"}), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
