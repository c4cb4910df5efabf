"""Generate tests/golden/explain_fold4.npz (data only) from the reference's bundled explanation files.

Run in the build container (reads /root/reference):  python tests/golden/make_explain_golden.py

  test_triples        explanation_datasets/test_filtered_fold4.csv (obj, rel, sbj), the test triples
                      all three explainers run on (explaiNE.py:59, GnnExplainer.py:101,
                      IDDGCN_explain.py:183)
  explaine_preds /    explanation_datasets/explaiNE_preds_fold4.npz as bundled (int64 / float32
  explaine_scores     arrays, loaded with allow_pickle=False).  They were produced with weights that
                      are not bundled (explaiNE.py:75 loads weights/new16180_1174_gcn_28_1754/...),
                      so they document the output format, not values the bundled weights reproduce.
  oracle_preds /      float64 oracle (oracle/ref_explain.explaine) on the bundled fold-4 weights for
  oracle_scores       the first 8 test triples: a regression pin of the oracle itself
The GNNExplainer / IDDGCN-explainer outputs and the ground truth ship as pickled object arrays; they
are not loaded (no unpickling of reference files).
"""
import os
import sys

import numpy as np
import pandas as pd

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))

from oracle import ref_explain  # noqa: E402

EX = "/root/reference/datasets/explanation_datasets"


def main():
    test = pd.read_csv(f"{EX}/test_filtered_fold4.csv").to_numpy().astype(np.int64)
    ref = np.load(f"{EX}/explaiNE_preds_fold4.npz", allow_pickle=False)
    d = np.load(os.path.join(HERE, "fold4_data.npz"))
    w = dict(np.load(os.path.join(HERE, "weights_fold4.npz")))
    adjacency = np.concatenate([d["X_train"].astype(np.int64), test])
    op, os_ = ref_explain.explaine(w, adjacency, test[:8], 845, 4, top_k=10)
    np.savez_compressed(os.path.join(HERE, "explain_fold4.npz"), test_triples=test,
                        explaine_preds=ref["preds"], explaine_scores=ref["scores"],
                        oracle_preds=op, oracle_scores=os_)


if __name__ == "__main__":
    main()
