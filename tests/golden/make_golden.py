"""Generate the committed golden fixtures under tests/golden/.

Run in the build container (needs /root/reference for the bundled data files):
    /opt/conda/bin/python3.9 oracle/convert_h5.py      # weights_fold{k}.npz
    python tests/golden/make_golden.py                   # everything below

Fixtures (all data, no code):
  fold{k}_data.npz   bundled fold files of the reference, as int arrays:
                     X_train (mode0_fold{k}_X_train.csv), X_test, neg_X_test,
                     X_train_neg (mode0_fold{k}_X_train_neg.npy, squeezed)
  fold{k}_eval.npz   oracle float64 eval probabilities and pre-sigmoid DistMult
                     logits on the bundled weights (IDDGCN_eval.py:49-122 with
                     fold=k; the same in float32 as probs32 / logits32, the
                     fp32 drift the parity bars are stated against), labels,
                     AUC/AUPR
  fold0_step.npz     one full train step on fold 0 from the bundled weights:
                     loss, scores, logits (float64 and float32), all parameter
                     gradients (float64 autograd of the reference op graph),
                     params after one Keras Adam step, layer outputs for the
                     first 256 scored edges (float64; float32 as layer*_32)
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

from oracle.ref_model import (KerasAdam, eval_metrics, forward_detail, predict,  # noqa: E402
                              train_step_grads)
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
        p64, s64 = predict(w, Xt, adj, N_ENT, dtype=torch.float64, logits=True)
        p32, s32 = predict(w, Xt, adj, N_ENT, dtype=torch.float32, logits=True)
        m = eval_metrics(y, p64)
        np.savez_compressed(os.path.join(HERE, f"fold{k}_eval.npz"), probs=p64, probs32=p32, logits=s64,
                            logits32=s32, y_true=y, roc_auc=m["roc_auc"], aupr=m["aupr"],
                            accuracy=m["accuracy"], f1=m["f1"])
        print(f"fold {k}: max|logit| {np.abs(s64).max():.2f}, fp32 logit drift {np.abs(s32 - s64).max():.2e}")
        print(f"fold {k}: auc {m['roc_auc']:.6f} aupr {m['aupr']:.6f}")

    # one training step on fold 0 from the bundled weights
    f = dict(np.load(os.path.join(HERE, "fold0_data.npz")))
    w = dict(np.load(os.path.join(HERE, "weights_fold0.npz")))
    adj = get_adj_coo(f["X_train"], N_ENT, N_REL)
    loss, scores, grads = train_step_grads(w, f["X_train"], f["X_train_neg"], adj, N_ENT)
    opt = KerasAdam()
    new = opt.step({k: v.astype(np.float64) for k, v in w.items()}, grads)
    scored = np.concatenate([f["X_train"], f["X_train_neg"]])
    _, s64, layers = forward_detail(w, scored, adj, N_ENT, dtype=torch.float64)
    _, s32, _ = forward_detail(w, scored, adj, N_ENT, dtype=torch.float32)
    _, _, layers32 = forward_detail(w, f["X_train"][:256], adj, N_ENT, dtype=torch.float32)
    out = {"loss": loss, "scores": scores, "logits": s64, "logits32": s32}
    out.update({f"grad_{k}": v for k, v in grads.items()})
    out.update({f"adam1_{k}": v for k, v in new.items()})
    for i, ((xh, xt), (xh32, xt32)) in enumerate(zip(layers, layers32), 1):
        out[f"layer{i}_head"] = xh[:256]
        out[f"layer{i}_tail"] = xt[:256]
        out[f"layer{i}_head32"] = xh32
        out[f"layer{i}_tail32"] = xt32
    print(f"fold0 step: max|logit| {np.abs(s64).max():.2f}, fp32 logit drift {np.abs(s32 - s64).max():.2e}")
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
    _, s64, layers = forward_detail(sp, np.concatenate([tri, neg]), adj, N, dtype=torch.float64)
    out = {"triples": tri, "neg": neg, "loss": loss, "scores": scores, "logits": s64, "N": N, "R": R, "D": D}
    for i, (xh, xt) in enumerate(layers, 1):
        out[f"layer{i}_head"] = xh
        out[f"layer{i}_tail"] = xt
    out.update({f"param_{k}": v for k, v in sp.items()})
    out.update({f"grad_{k}": v for k, v in grads.items()})
    out.update({f"adam1_{k}": v for k, v in new.items()})
    np.savez_compressed(os.path.join(HERE, "synth_small.npz"), **out)
    print("synth loss", loss)


if __name__ == "__main__":
    main()
