"""Generate the committed golden fixtures under tests/golden/.

Run in the build container (needs /root/reference for the bundled data files):
    /opt/conda/bin/python3.9 oracle/convert_h5.py      # weights_fold{k}.npz
    python tests/golden/make_golden.py                   # everything below

Fixtures (all data, no code):
  fold{k}_data.npz   bundled fold files of the reference, as int arrays:
                     X_train (mode0_fold{k}_X_train.csv), X_test, neg_X_test,
                     X_train_neg (mode0_fold{k}_X_train_neg.npy, squeezed)
  fold{k}_eval.npz   oracle float64 eval probabilities on the bundled weights
                     (IDDGCN_eval.py:49-122 with fold=k), labels, AUC/AUPR
  fold0_step.npz     one full train step on fold 0 from the bundled weights:
                     loss, scores, all parameter gradients (float64 autograd
                     of the reference op graph), params after one Keras Adam
                     step, layer outputs for the first 256 scored edges
  synth_small.npz    a small synthetic graph (N=512, D=32, R=2) with the same
                     quantities at a non-saturating init
"""
import os
import sys

import numpy as np
import pandas as pd
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))

from oracle.ref_model import (KerasAdam, adj_to_torch, eval_metrics, model_forward,  # noqa: E402
                              predict, to_torch_params, train_step_grads)
from oracle.ref_utils import get_adj_coo, get_y_true, make_fold_files  # noqa: E402

DATA = "/root/reference/datasets/prediction_datasets"
N_ENT, N_REL = 845, 4


def fold_data(k):
    f = {
        "X_train": pd.read_csv(f"{DATA}/mode0_fold{k}_X_train.csv").to_numpy().astype(np.int32),
        "X_test": pd.read_csv(f"{DATA}/mode0_fold{k}_X_test.csv").to_numpy().astype(np.int32),
        "neg_X_test": pd.read_csv(f"{DATA}/mode0_fold{k}_neg_X_test.csv", index_col=0).to_numpy().astype(np.int32),
        "X_train_neg": np.load(f"{DATA}/mode0_fold{k}_X_train_neg.npy")[0].astype(np.int32),
    }
    # pin: the oracle's split restatement reproduces the bundled files bit-for-bit
    re = make_fold_files(DATA, k)
    for name in f:
        a = re[name][0] if name == "X_train_neg" else re[name]
        assert np.array_equal(a.astype(np.int64), f[name].astype(np.int64)), (k, name)
    return f


def main():
    for k in range(5):
        f = fold_data(k)
        np.savez_compressed(os.path.join(HERE, f"fold{k}_data.npz"), **f)
        w = dict(np.load(os.path.join(HERE, f"weights_fold{k}.npz")))
        adj = get_adj_coo(np.concatenate([f["X_train"], f["X_test"]]), N_ENT, N_REL)
        Xt = np.concatenate([f["X_test"], f["neg_X_test"]]).astype(np.int64)
        y = get_y_true(f["X_test"], Xt)
        p64 = predict(w, Xt, adj, N_ENT, dtype=torch.float64)
        p32 = predict(w, Xt, adj, N_ENT, dtype=torch.float32)
        m = eval_metrics(y, p64)
        np.savez_compressed(os.path.join(HERE, f"fold{k}_eval.npz"), probs=p64, probs32=p32, y_true=y,
                            roc_auc=m["roc_auc"], aupr=m["aupr"], accuracy=m["accuracy"], f1=m["f1"])
        print(f"fold {k}: auc {m['roc_auc']:.6f} aupr {m['aupr']:.6f}")

    # one training step on fold 0 from the bundled weights
    f = dict(np.load(os.path.join(HERE, "fold0_data.npz")))
    w = dict(np.load(os.path.join(HERE, "weights_fold0.npz")))
    adj = get_adj_coo(f["X_train"], N_ENT, N_REL)
    loss, scores, grads = train_step_grads(w, f["X_train"], f["X_train_neg"], adj, N_ENT)
    opt = KerasAdam()
    new = opt.step({k: v.astype(np.float64) for k, v in w.items()}, grads)
    P = to_torch_params(w, torch.float64, requires_grad=False)
    tr = f["X_train"][:256].astype(np.int64)
    with torch.no_grad():
        _, layers = model_forward(P, tr[:, 0], tr[:, 1], tr[:, 2], adj_to_torch(adj, N_ENT), return_layers=True)
    out = {"loss": loss, "scores": scores}
    out.update({f"grad_{k}": v for k, v in grads.items()})
    out.update({f"adam1_{k}": v for k, v in new.items()})
    for i, (xh, xt) in enumerate(layers, 1):
        out[f"layer{i}_head"] = xh.numpy()
        out[f"layer{i}_tail"] = xt.numpy()
    np.savez_compressed(os.path.join(HERE, "fold0_step.npz"), **out)
    print("fold0 step loss", loss)

    # small synthetic graph at a non-saturating init
    rng = np.random.default_rng(0)
    N, R, D = 512, 2, 32
    pairs = set()
    while len(pairs) < 1500:
        a, b = rng.integers(0, N, 2)
        if a != b:
            pairs.add((min(a, b), max(a, b)))
    pairs = np.array(sorted(pairs))
    rel = rng.integers(0, R, len(pairs))
    tri = np.concatenate([np.stack([pairs[:, 0], rel, pairs[:, 1]], 1),
                          np.stack([pairs[:, 1], rel, pairs[:, 0]], 1)]).astype(np.int32)
    rng.shuffle(tri)
    neg = tri[: len(tri) // 2].copy()
    flip = rng.integers(0, 2, len(neg)).astype(bool)
    rnd = rng.integers(0, N, len(neg))
    neg[flip, 0] = rnd[flip]
    neg[~flip, 2] = rnd[~flip]
    sp = {"E": rng.standard_normal((N, D)) / np.sqrt(D)}
    for l in (1, 2, 3):
        sp[f"K{l}"] = rng.standard_normal((R, D, D)) / np.sqrt(D)
        sp[f"S{l}"] = rng.standard_normal((D, D)) / np.sqrt(D)
        sp[f"relw{l}"] = rng.uniform(-0.05, 0.05, R)
        sp[f"Wa{l}"] = rng.standard_normal((D, R)) / np.sqrt(D)
        sp[f"ba{l}"] = rng.standard_normal(R) * 0.1
    sp["rel"] = rng.standard_normal((R, D))
    sp = {k: v.astype(np.float32) for k, v in sp.items()}
    adj = get_adj_coo(tri, N, R)
    loss, scores, grads = train_step_grads(sp, tri, neg, adj, N)
    opt = KerasAdam()
    new = opt.step({k: v.astype(np.float64) for k, v in sp.items()}, grads)
    out = {"triples": tri, "neg": neg, "loss": loss, "scores": scores, "N": N, "R": R, "D": D}
    out.update({f"param_{k}": v for k, v in sp.items()})
    out.update({f"grad_{k}": v for k, v in grads.items()})
    out.update({f"adam1_{k}": v for k, v in new.items()})
    np.savez_compressed(os.path.join(HERE, "synth_small.npz"), **out)
    print("synth loss", loss)


if __name__ == "__main__":
    main()
