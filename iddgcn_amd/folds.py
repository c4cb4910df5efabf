"""The reference's fold construction (prediction/utils1.py:741-867, IDDGCN.py:312-373), host side.

Data preparation around the hot path, done once per run on a few thousand triples, so it stays
numpy/pandas on the host like the reference; the row orders it produces ARE the scored-edge and
adjacency inputs of training, so they are reproduced exactly (the bundled fold files are the check,
tests/test_folds.py):

* ``shuffled(df, seed)``: DataFrame.sample(frac=1, random_state=seed) (and sklearn's shuffle) is the
  legacy RandomState(seed).permutation of the rows;
* ``kfold_ranges``: sklearn KFold(n) without shuffling — contiguous test ranges, the first n % k
  folds one row longer, train = the other rows in order;
* modes 1-3 (cold-start splits by mutation / drug id ranges) select rows by node membership; the
  reference's left-merge-and-drop is, for rows drawn from the same frame, the complement mask.
"""
import numpy as np
import pandas as pd

COLS = ["obj", "rel", "sbj"]


def shuffled(df, seed):
    """df.sample(frac=1, random_state=seed).reset_index(drop=True)."""
    return df.iloc[np.random.RandomState(seed).permutation(len(df))].reset_index(drop=True)


def kfold_ranges(n, k):
    """[(train_idx, test_idx)] of sklearn.model_selection.KFold(n_splits=k).split on n rows."""
    if not 2 <= k <= max(n, 2):
        raise ValueError(f"cannot split {n} rows into {k} folds")
    sizes = np.full(k, n // k, dtype=np.int64)
    sizes[: n % k] += 1
    bounds = np.concatenate([[0], np.cumsum(sizes)])
    idx = np.arange(n)
    return [(np.concatenate([idx[:a], idx[b:]]), idx[a:b]) for a, b in zip(bounds[:-1], bounds[1:])]


def _touches(df, nodes):
    nodes = np.asarray(list(nodes), dtype=np.int64)
    return np.isin(df["obj"].to_numpy(), nodes) | np.isin(df["sbj"].to_numpy(), nodes)


def _cold_split(frame, nodes, new_node_split):
    """Rows touching ``nodes`` -> test, the others -> train; with ``new_node_split`` (mode 3) the other
    endpoints of the test rows are halved between the two sides (utils1.py:778-804, 841-865)."""
    hit = _touches(frame, nodes)
    test, train = frame[hit], frame[~hit].reset_index(drop=True)
    if new_node_split:
        others = np.setdiff1d(np.unique(test[["obj", "sbj"]].to_numpy()), np.asarray(list(nodes)))
        half = len(others) // 2
        to_test, to_train = others[:half], others[half:]
        test = test[~_touches(test, to_test)]
        train = train[~_touches(train, to_train)]
    return train.astype(int), test.astype(int)


def split_pos_triple_into_folds(dc, cc, dd, num_folds, seed, mode):
    """utils1.split_pos_triple_into_folds: response triples ``dc`` split into folds, similarity
    triples ``cc`` / ``dd`` always in training.  Returns [(train_df, test_df)] per fold."""
    dc, cc, dd = shuffled(dc, seed), shuffled(cc, seed), shuffled(dd, seed)
    if mode == 0:
        sims = pd.concat([cc, dd], axis=0)
        return [(pd.concat([dc.iloc[tr], sims], axis=0), dc.iloc[te]) for tr, te in kfold_ranges(len(dc), num_folds)]
    allt = pd.concat([dc, dd, cc], axis=0).astype(int)
    out = []
    for i in range(num_folds):
        if mode == 1:
            w = 660 // num_folds
            nodes = range(w * i, w * (i + 1))
        elif mode == 2:
            w = 157 / num_folds
            nodes = range(int(w * i + 660), int(w * (i + 1) + 660))
        else:
            w = 660 / num_folds
            nodes = range(int(w * i), int(w * (i + 1)))
        out.append(_cold_split(allt, nodes, mode not in (1, 2)))
    return out


def split_neg_triple_into_folds(dc, num_folds, seed, mode):
    """utils1.split_neg_triple_into_folds (no shuffling of the negatives)."""
    if mode == 0:
        return [(dc.iloc[tr], dc.iloc[te]) for tr, te in kfold_ranges(len(dc), num_folds)]
    out = []
    for i in range(num_folds):
        if mode == 1:
            w = 477 // num_folds
            nodes = range(w * i, w * (i + 1))
        elif mode == 2:
            w = 157 / num_folds
            nodes = range(int(w * i + 477), int(w * (i + 1) + 477))
        else:
            w = 477 / num_folds
            nodes = range(int(w * i), int(w * (i + 1)))
        out.append(_cold_split(dc, nodes, mode not in (1, 2)))
    return out


def reverse_triples(df):
    """utils1.generate_reverse_triplets as a frame: (sbj, rel, obj) of every row with obj != sbj."""
    a = df.to_numpy()
    a = a[a[:, 0] != a[:, 2]][:, [2, 1, 0]]
    return pd.DataFrame(a, columns=COLS)


def make_fold(data_dir, fold, mode=0, seed=89, num_splits=5):
    """IDDGCN.py:312-373 for one (mode, fold): the arrays the training script writes and trains on —
    X_train (response + similarity triples + reverses), X_test (response test triples + reverses),
    neg_X_test (test negatives of relations 0/1), X_train_neg (training negatives + reverses, (1, n, 3))."""
    resp = pd.read_csv(f"{data_dir}/triplets_dc.csv", header=0)
    resp = resp.iloc[np.random.RandomState(24).permutation(len(resp))]       # sklearn shuffle(random_state=24)
    mu = pd.read_csv(f"{data_dir}/mu_similar0.97.csv", header=0)
    dr = pd.read_csv(f"{data_dir}/drug_similar0.78.csv", header=0)
    neg = pd.read_csv(f"{data_dir}/negative_dc_28_1754.csv", header=0)
    for df in (resp, mu, dr):
        df.columns = COLS
    neg.columns = COLS
    tr_pos, te_pos = split_pos_triple_into_folds(resp, mu, dr, num_splits, seed, mode)[fold]
    tr_neg, te_neg = split_neg_triple_into_folds(neg, num_splits, seed, mode)[fold]
    te_neg_f = te_neg[te_neg["rel"].isin([0, 1])]
    # IDDGCN.py:344 drops the rel 2/3 test rows BY INDEX LABEL: in the cold-start modes the test frame keeps
    # the repeated labels of concat([dc, dd, cc]), so response rows sharing a label with one go too
    te_pos = te_pos.drop(te_pos[te_pos["rel"].isin([2, 3])].index)
    X_train = pd.concat([tr_pos, reverse_triples(tr_pos)], axis=0).astype(np.int64)
    X_test = pd.concat([te_pos, reverse_triples(te_pos)], axis=0).astype(np.int64)
    X_train_neg = pd.concat([tr_neg, reverse_triples(tr_neg)], axis=0)
    return {"X_train": X_train.to_numpy(), "X_test": X_test.to_numpy(), "neg_X_test": te_neg_f.to_numpy(),
            "X_train_neg": np.expand_dims(X_train_neg.to_numpy(), 0)}
