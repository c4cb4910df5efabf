"""Convert the reference's Keras-h5 weight files to .npz fixtures.

TEST INFRASTRUCTURE ONLY.  Runs under the image's secondary interpreter that
has h5py (``/opt/conda/bin/python3.9 oracle/convert_h5.py``); h5py only reads
datasets (no pickle, nothing executed from the file).

Keras ``load_weights`` on an h5 file is positional over the layers that own
weights, in the order of the file's ``layer_names`` attribute
(IDDGCN_eval.py:46-47).  For this model that order is
entity_embeddings, layer1, layer2, layer3, DistMult, and each IDDGCN layer
stores [relation_kernels, self_kernel, relation_weights, W_alpha, b_alpha]
(IDDGCN.py:25-58).
"""
import os
import sys

import h5py
import numpy as np

REF = "/root/reference/datasets/prediction_datasets/weights/IDDGCN_normal"
NAME = "mode0_fold{k}_epoch5000_learnRate0.001_batchsize100_embdim64_weight.h5"


def convert(path):
    f = h5py.File(path, "r")
    names = [n.decode() if isinstance(n, bytes) else str(n) for n in f.attrs["layer_names"]]
    weighted = []
    for n in names:
        wn = f[n].attrs["weight_names"]
        if len(wn):
            weighted.append([np.asarray(f[n][w.decode() if isinstance(w, bytes) else str(w)]) for w in wn])
    assert len(weighted) == 5, [len(w) for w in weighted]
    out = {"E": weighted[0][0]}
    for l in (1, 2, 3):
        K, S, relw, Wa, ba = weighted[l]
        out.update({f"K{l}": K, f"S{l}": S, f"relw{l}": relw, f"Wa{l}": Wa, f"ba{l}": ba})
    out["rel"] = weighted[4][0]
    return {k: v.astype(np.float32) for k, v in out.items()}


if __name__ == "__main__":
    dst = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(__file__), "..", "tests", "golden")
    for k in range(5):
        w = convert(os.path.join(REF, NAME.format(k=k)))
        np.savez_compressed(os.path.join(dst, f"weights_fold{k}.npz"), **w)
        print(k, {n: a.shape for n, a in w.items()})
