"""tests/golden/similarity.npz: the inputs and outputs of prediction/feat_similarity.py.

Run in the build container (needs /root/reference):  python tests/golden/make_similarity_golden.py
  mu_feat   (661, 248) float64  Mutation_feature_248.csv (index column dropped)
  drug_feat (184, 248) float64  drug_feature_248.csv, NaN rows dropped (feat_similarity.py:8)
  mu_triples / drug_triples     the reference's own outputs mu_similar0.97.csv / drug_similar0.78.csv
"""
import os
import sys

import numpy as np
import pandas as pd

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
from oracle.ref_similarity import similar_triples  # noqa: E402

DATA = "/root/reference/datasets/prediction_datasets"


def main():
    mu = pd.read_csv(f"{DATA}/Mutation_feature_248.csv", header=None, index_col=0).to_numpy(np.float64)
    drug = pd.read_csv(f"{DATA}/drug_feature_248.csv", header=None, index_col=0).dropna().to_numpy(np.float64)
    mu_t = pd.read_csv(f"{DATA}/mu_similar0.97.csv", header=None).to_numpy(np.int64)
    drug_t = pd.read_csv(f"{DATA}/drug_similar0.78.csv", header=None).to_numpy(np.int64)
    assert np.array_equal(similar_triples(mu, 0.97, 3, 0), mu_t)          # the oracle is pinned
    assert np.array_equal(similar_triples(drug, 0.78, 2, len(mu)), drug_t)
    np.savez_compressed(os.path.join(HERE, "similarity.npz"), mu_feat=mu, drug_feat=drug, mu_triples=mu_t,
                        drug_triples=drug_t)


if __name__ == "__main__":
    main()
