"""Keras-h5 weight IO without h5py (iddgcn_amd/h5lite.py).

* reader: the reference's five bundled weight files (read where /root/reference exists) equal the
  committed npz fixtures, which were converted with h5py (oracle/convert_h5.py);
* writer: save_weights(.h5) round-trips through the reader; when the image's secondary interpreter
  with h5py is present, h5py reads the written file back identically (the file is real HDF5).
"""
import os
import subprocess
import sys

import numpy as np
import pytest

from iddgcn_amd import get_IDDGCN_Model, h5lite
from iddgcn_amd.weights_io import NAMES, load_h5

REF_W = "/root/reference/datasets/prediction_datasets/weights/IDDGCN_normal"
H5PY_PY = "/opt/conda/bin/python3.9"


@pytest.mark.skipif(not os.path.isdir(REF_W), reason="reference weight files only in the build container")
@pytest.mark.parametrize("k", range(5))
def test_reader_matches_h5py_conversion(k, golden):
    w = load_h5(os.path.join(REF_W, f"mode0_fold{k}_epoch5000_learnRate0.001_batchsize100_embdim64_weight.h5"))
    g = golden(f"weights_fold{k}.npz")
    for n in NAMES:
        assert np.array_equal(w[n], g[n]), n


@pytest.mark.skipif(not os.path.isdir(REF_W), reason="reference weight files only in the build container")
def test_reader_structure_and_attributes():
    f = h5lite.open_file(os.path.join(REF_W, "mode0_fold0_epoch5000_learnRate0.001_batchsize100_embdim64_weight.h5"))
    assert f.attrs["keras_version"] == "2.7.0" and f.attrs["backend"] == "tensorflow"
    names = list(f.attrs["layer_names"])
    assert names[:4] == ["all_entities", "head_input", "tail_input", "entity_embeddings"]
    assert list(f["rgcn__layer"].attrs["weight_names"]) == ["relation_kernels:0", "self_kernel:0",
                                                             "relation_weights:0", "W_alpha:0", "b_alpha:0"]
    assert np.asarray(f["entity_embeddings/entity_embeddings/embeddings:0"]).shape == (845, 64)
    with pytest.raises(KeyError):
        f["no_such_layer"]


def _model(golden, tmp):
    m = get_IDDGCN_Model(845, 4, 64, 64, 1, None, 0, 0)
    w = golden("weights_fold0.npz")
    m._set_named({k: w[k] for k in NAMES})
    return m


def test_writer_round_trip(golden, tmp_path):
    m = _model(golden, tmp_path)
    p = str(tmp_path / "w.h5")
    m.save_weights(p)
    with open(p, "rb") as f:
        assert f.read(8) == b"\x89HDF\r\n\x1a\n"
    back = load_h5(p)
    w = golden("weights_fold0.npz")
    for n in NAMES:
        assert np.array_equal(back[n], w[n]), n
    m2 = get_IDDGCN_Model(845, 4, 64, 64, 2, None, 0, 0)
    m2.load_weights(p)
    for a, b in zip(m2.get_weights(), m.get_weights()):
        assert np.array_equal(a, b)


@pytest.mark.skipif(not os.path.exists(H5PY_PY), reason="no h5py interpreter in this image")
def test_written_file_reads_in_h5py(golden, tmp_path):
    m = _model(golden, tmp_path)
    p = str(tmp_path / "w.h5")
    m.save_weights(p)
    code = ("import h5py, numpy as np, sys\n"
            "f = h5py.File(sys.argv[1], 'r')\n"
            "names = [n.decode() for n in f.attrs['layer_names']]\n"
            "out = {}\n"
            "for n in names:\n"
            "    for w in f[n].attrs['weight_names']:\n"
            "        out[n + '|' + w.decode()] = np.asarray(f[n][w.decode()])\n"
            "np.savez(sys.argv[2], **out)\n"
            "print(names, f.attrs['keras_version'])\n")
    out = str(tmp_path / "back.npz")
    env = {k: v for k, v in os.environ.items() if k not in ("PYTHONPATH", "PYTHONHOME")}
    r = subprocess.run([H5PY_PY, "-c", code, p, out], capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode == 0, r.stderr
    back = dict(np.load(out))
    w = golden("weights_fold0.npz")
    assert np.array_equal(back["entity_embeddings|entity_embeddings/embeddings:0"], w["E"])
    assert np.array_equal(back["DistMult|DistMult/rel_embedding:0"], w["rel"])
    assert np.array_equal(back["iddgcn__layer_2|self_kernel:0"], w["S3"])
    assert np.array_equal(back["iddgcn__layer|relation_kernels:0"], w["K1"])
