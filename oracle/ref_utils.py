"""numpy/pandas restatement of the data/graph helpers of the reference.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).  Each function cites the
reference function it restates; the reference module itself cannot be
imported here because it imports tensorflow at ``prediction/utils1.py:4``.
"""
import numpy as np
import pandas as pd
from sklearn.model_selection import KFold


def distinct(a):
    """utils1.py:415-417 — lexicographically sorted unique rows."""
    return np.unique(np.asarray(a), axis=0)


def get_adj_coo(data, num_entities, num_relations):
    """utils1.py:420-451 (get_adj_mats) without TensorFlow.

    Returns a list of ``(indices[int64, nnz x 2], values[float32, nnz])`` per
    relation, in the order ``tf.sparse.reorder`` leaves them (row-major sorted).
    An empty relation yields the single placeholder entry (0,0)=0.0 exactly as
    utils1.py:427-429 does.
    """
    data = np.asarray(data)
    out = []
    for i in range(num_relations):
        data_i = data[data[:, 1] == i]
        if not data_i.shape[0]:
            idx = np.zeros((1, 2), dtype=np.int64)
            val = np.zeros((1,), dtype=np.float32)
        else:
            idx = distinct(data_i[:, [0, 2]]).astype(np.int64)
            val = np.ones((idx.shape[0],), dtype=np.float32)
        # tf.sparse.reorder: row-major order; np.unique already provides it.
        order = np.lexsort((idx[:, 1], idx[:, 0]))
        out.append((idx[order], val[order]))
    return out


def generate_reverse_triplets(triplets):
    """utils1.py:616-623 — (t, r, h) for every triple with h != t."""
    rev = [(t, r, h) for h, r, t in np.asarray(triplets).tolist() if h != t]
    return np.array(rev)


def generate_negative_samples_np(heads, relations, tails, num_entities, seed):
    """utils1.py:646-655 — corrupt head or tail with a uniform entity."""
    np.random.seed(seed)
    cond = np.random.randint(0, 2, size=heads.shape)
    rnd = np.random.randint(0, num_entities, size=heads.shape)
    neg_heads = np.where(cond == 0, heads, rnd)
    neg_tails = np.where(cond == 1, tails, rnd)
    return neg_heads, relations, neg_tails


def get_y_true(X_test_pos, X_test_rule):
    """utils1.py:657-663 — 1 where a scored triple is a test positive."""
    pos = pd.DataFrame(X_test_pos).drop_duplicates()
    rule = pd.DataFrame(X_test_rule)
    merged = pd.merge(rule, pos, indicator=True, how='left')
    return (merged['_merge'] == 'both').astype(int).values


def _merge_left_only(frame, sub):
    """pd.merge(frame, sub, how='left', indicator=True) rows marked 'left_only', as the reference
    computes the training side of its cold-start splits (utils1.py:767-769)."""
    m = pd.merge(frame, sub, how='left', indicator=True)
    return m[m['_merge'] == 'left_only'].drop('_merge', axis=1).astype(int)


def _cold_fold(frame, nodes, mode3):
    """utils1.py:762-804 / 817-865 for one fold: rows touching ``nodes`` are the test side; mode 3 then
    halves the other endpoints of those rows between test and train."""
    pre_test = frame[(frame['obj'].isin(nodes)) | (frame['sbj'].isin(nodes))]
    pre_train = _merge_left_only(frame, pre_test)
    if not mode3:
        return pre_train, pre_test.astype(int)
    new_node = list(np.setdiff1d(np.unique(pre_test[['obj', 'sbj']].values), nodes))
    nt, ntr = new_node[:len(new_node) // 2], new_node[len(new_node) // 2:]
    test = pre_test[~pre_test['obj'].isin(nt) & ~pre_test['sbj'].isin(nt)].astype(int)
    train = pre_train[~pre_train['obj'].isin(ntr) & ~pre_train['sbj'].isin(ntr)].astype(int)
    return train, test


def split_pos_triple_into_folds(dc, cc, dd, num_folds, seed, mode=0):
    """utils1.py:741-807 (all four modes)."""
    dc = dc.sample(frac=1, random_state=seed).reset_index(drop=True)
    cc = cc.sample(frac=1, random_state=seed).reset_index(drop=True)
    dd = dd.sample(frac=1, random_state=seed).reset_index(drop=True)
    if mode == 0:
        cc_dd = pd.concat([cc, dd], axis=0)
        splits = []
        for tr, te in KFold(n_splits=num_folds).split(dc):
            splits.append((pd.concat([dc.iloc[tr], cc_dd], axis=0), dc.iloc[te]))
        return splits
    allt = pd.concat([dc, dd, cc], axis=0).astype(int)
    out = []
    for i in range(num_folds):
        if mode == 1:
            lf = 660 // num_folds
            nodes = range(int(lf * i), int(lf * (i + 1)))
        elif mode == 2:
            lf = 157 / num_folds
            nodes = range(int(lf * i + 660), int(lf * (i + 1) + 660))
        else:
            lf = 660 / num_folds
            nodes = range(int(lf * i), int(lf * (i + 1)))
        out.append(_cold_fold(allt, nodes, mode not in (1, 2)))
    return out


def split_neg_triple_into_folds(dc, num_folds, seed, mode=0):
    """utils1.py:808-867 (all four modes)."""
    if mode == 0:
        return [(dc.iloc[tr], dc.iloc[te]) for tr, te in KFold(n_splits=num_folds).split(dc)]
    out = []
    for i in range(num_folds):
        if mode == 1:
            lf = 477 // num_folds
            nodes = range(int(lf * i), int(lf * (i + 1)))
        elif mode == 2:
            lf = 157 / num_folds
            nodes = range(int(lf * i + 477), int(lf * (i + 1) + 477))
        else:
            lf = 477 / num_folds
            nodes = range(int(lf * i), int(lf * (i + 1)))
        out.append(_cold_fold(dc, nodes, mode not in (1, 2)))
    return out


def make_fold_files(data_dir, fold, seed=89, num_splits=5, mode=0):
    """IDDGCN.py:312-373 — rebuild one fold's X_train / X_test / neg files.

    Returns dict of numpy arrays equal to the bundled
    ``mode0_fold{k}_X_train.csv``, ``_X_test.csv``, ``_neg_X_test.csv`` and
    ``_X_train_neg.npy`` (the survey verified bit-for-bit reproduction).  ``mode`` 1-3 runs the same
    script body on the cold-start splits (IDDGCN.py:327 loops mode over range(0, 1) only); the test-side
    drop of rel 2/3 rows is the script's label-based DataFrame.drop (:344), which in these modes also
    removes response rows sharing a label with a dropped row (the cold-start test frames keep the
    repeated labels of concat([dc, dd, cc])).
    """
    from sklearn.utils import shuffle
    resp = pd.read_csv(f"{data_dir}/triplets_dc.csv", header=0)
    resp = shuffle(resp, random_state=24)
    mu = pd.read_csv(f"{data_dir}/mu_similar0.97.csv", header=0)
    dr = pd.read_csv(f"{data_dir}/drug_similar0.78.csv", header=0)
    neg = pd.read_csv(f"{data_dir}/negative_dc_28_1754.csv", header=0)
    for df in (resp, mu, dr):
        df.columns = ['obj', 'rel', 'sbj']
    pos_splits = split_pos_triple_into_folds(resp, mu, dr, num_splits, seed, mode)
    neg_splits = split_neg_triple_into_folds(neg, num_splits, seed, mode)
    X_train_t, X_test_t = pos_splits[fold]
    neg_train, neg_test = neg_splits[fold]
    neg_test_f = neg_test[neg_test['rel'].isin([0, 1])]
    X_test_t = X_test_t.drop(X_test_t[(X_test_t['rel'] == 2) | (X_test_t['rel'] == 3)].index)
    syn_tr = pd.DataFrame(generate_reverse_triplets(X_train_t.to_numpy()), columns=['obj', 'rel', 'sbj'])
    syn_neg_tr = pd.DataFrame(generate_reverse_triplets(neg_train.to_numpy()), columns=['obj', 'rel', 'sbj'])
    syn_te = pd.DataFrame(generate_reverse_triplets(X_test_t.to_numpy()), columns=['obj', 'rel', 'sbj'])
    neg_train_all = pd.concat([neg_train, syn_neg_tr], axis=0)
    X_train = pd.concat([X_train_t, syn_tr], axis=0).astype(np.int64)
    X_test = pd.concat([X_test_t, syn_te], axis=0).astype(np.int64)
    return {
        'X_train': X_train.to_numpy(),
        'X_test': X_test.to_numpy(),
        'neg_X_test': neg_test_f.to_numpy(),
        'X_train_neg': np.expand_dims(neg_train_all.to_numpy(), 0),
    }
