"""The product's fold construction (iddgcn_amd/folds.py) against the oracle's restatement of
utils1.py:741-867 (pandas merges, sklearn KFold) in all four modes, and — mode 0 — against the
reference's bundled fold files (tests/golden/fold{k}_data.npz, themselves reproduced bit-for-bit by
the oracle, tests/test_oracle.py)."""
import os

import numpy as np
import pandas as pd
import pytest

from iddgcn_amd import folds
from oracle import ref_utils
from tests.conftest import REFERENCE


def _frames(rng, n_resp=400, n_sim=300, n_neg=350):
    def tri(n, hi_a, hi_b, rels):
        return pd.DataFrame({"obj": rng.integers(0, hi_a, n), "rel": rng.choice(rels, n),
                             "sbj": rng.integers(hi_a, hi_a + hi_b, n)})
    dc = tri(n_resp, 660, 185, [0, 1])
    cc = pd.DataFrame({"obj": rng.integers(0, 660, n_sim), "rel": 3, "sbj": rng.integers(0, 660, n_sim)})
    dd = pd.DataFrame({"obj": rng.integers(660, 845, n_sim // 4), "rel": 2, "sbj": rng.integers(660, 845, n_sim // 4)})
    neg = pd.DataFrame({"obj": rng.integers(0, 660, n_neg), "rel": rng.choice([0, 1], n_neg),
                        "sbj": rng.integers(0, 660, n_neg)})
    return dc, cc, dd, neg


def test_kfold_ranges_match_sklearn():
    from sklearn.model_selection import KFold
    for n in (5, 7, 1754, 2806):
        for k in (2, 3, 5):
            ours = folds.kfold_ranges(n, k)
            ref = list(KFold(n_splits=k).split(np.arange(n)))
            assert len(ours) == len(ref)
            for (a, b), (c, d) in zip(ours, ref):
                assert np.array_equal(a, c) and np.array_equal(b, d)


def test_shuffle_is_pandas_sample():
    df = pd.DataFrame({"a": np.arange(1000)})
    assert np.array_equal(folds.shuffled(df, 89)["a"].to_numpy(),
                          df.sample(frac=1, random_state=89).reset_index(drop=True)["a"].to_numpy())


@pytest.mark.parametrize("mode", [0, 1, 2, 3])
def test_splits_match_oracle_all_modes(mode):
    dc, cc, dd, neg = _frames(np.random.default_rng(mode))
    ours = folds.split_pos_triple_into_folds(dc, cc, dd, 5, 89, mode)
    ref = ref_utils.split_pos_triple_into_folds(dc, cc, dd, 5, 89, mode)
    ours_n = folds.split_neg_triple_into_folds(neg, 5, 89, mode)
    ref_n = ref_utils.split_neg_triple_into_folds(neg, 5, 89, mode)
    for (a, b), (c, d) in list(zip(ours, ref)) + list(zip(ours_n, ref_n)):
        assert np.array_equal(a.to_numpy(), c.to_numpy())
        assert np.array_equal(b.to_numpy(), d.to_numpy())


@pytest.mark.skipif(not os.path.isdir(REFERENCE), reason="reference datasets not present")
@pytest.mark.parametrize("k", range(5))
def test_make_fold_reproduces_bundled_files(k, golden):
    f = golden(f"fold{k}_data.npz")
    ours = folds.make_fold(REFERENCE, k)
    for name in ("X_train", "X_test", "neg_X_test"):
        assert np.array_equal(ours[name].astype(np.int64), f[name].astype(np.int64)), name
    assert np.array_equal(ours["X_train_neg"][0].astype(np.int64), f["X_train_neg"].astype(np.int64))


@pytest.mark.skipif(not os.path.isdir(REFERENCE), reason="reference datasets not present")
@pytest.mark.parametrize("mode", [1, 2, 3])
def test_make_fold_cold_start_modes_follow_the_script(mode):
    """Modes 1-3 (IDDGCN.py:312-363 with mode != 0): the product's make_fold equals the oracle's restatement
    of the script body, including the label-based drop of the rel 2/3 test rows (:344) that also removes
    response rows whose label repeats one of theirs."""
    for k in range(5):
        ours = folds.make_fold(REFERENCE, k, mode=mode)
        ref = ref_utils.make_fold_files(REFERENCE, k, mode=mode)
        for name in ("X_train", "X_test", "neg_X_test", "X_train_neg"):
            assert np.array_equal(ours[name].astype(np.int64), ref[name].astype(np.int64)), (mode, k, name)
