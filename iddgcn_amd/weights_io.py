"""Weight files: the repo's .npz layout and (when h5py is importable) Keras h5.

Keras ``load_weights`` on an h5 file is positional over the layers that own
weights, in the order of the file's ``layer_names`` attribute
(IDDGCN_eval.py:46-47): entity_embeddings, the three IDDGCN layers
([relation_kernels, self_kernel, relation_weights, W_alpha, b_alpha] each,
IDDGCN.py:25-58), DistMult [rel_embedding].  The .npz layout uses the names
E, K1, S1, relw1, Wa1, ba1, ..., rel (tests/golden/weights_fold*.npz are the
reference's bundled h5 files converted to it).
"""
import numpy as np

NAMES = ["E"] + [f"{k}{l}" for l in (1, 2, 3) for k in ("K", "S", "relw", "Wa", "ba")] + ["rel"]


def load_any(path, model=None):
    if path.endswith(".h5"):
        return load_h5(path)
    with np.load(path, allow_pickle=False) as z:
        missing = [n for n in NAMES if n not in z.files]
        if missing:
            raise ValueError(f"{path}: missing arrays {missing}")
        return {n: np.asarray(z[n], dtype=np.float32) for n in NAMES}


def load_h5(path):
    try:
        import h5py
    except ImportError as e:
        raise ImportError("reading Keras .h5 weights needs h5py; convert with oracle/convert_h5.py "
                          "or pass the .npz layout") from e
    with h5py.File(path, "r") as f:
        dec = lambda s: s.decode() if isinstance(s, bytes) else str(s)  # noqa: E731
        weighted = []
        for n in (dec(x) for x in f.attrs["layer_names"]):
            wn = [dec(w) for w in f[n].attrs["weight_names"]]
            if wn:
                weighted.append([np.asarray(f[n][w], dtype=np.float32) for w in wn])
    if len(weighted) != 5:
        raise ValueError(f"{path}: expected 5 weighted layers, found {len(weighted)}")
    out = {"E": weighted[0][0], "rel": weighted[4][0]}
    for l in (1, 2, 3):
        for k, a in zip(("K", "S", "relw", "Wa", "ba"), weighted[l]):
            out[f"{k}{l}"] = a
    return out


def save_h5(path, model):
    import h5py
    d = model._named()
    names = ["entity_embeddings"] + [l.name for l in model.gcn_layers] + ["DistMult"]
    with h5py.File(path, "w") as f:
        f.attrs["layer_names"] = np.array([n.encode() for n in names])
        f.attrs["backend"] = b"tensorflow"
        f.attrs["keras_version"] = b"2.7.0"
        groups = [("entity_embeddings", [("embeddings:0", d["E"])])]
        for i, l in enumerate(model.gcn_layers, 1):
            groups.append((l.name, [(f"{w}:0", d[k]) for w, k in zip(
                ("relation_kernels", "self_kernel", "relation_weights", "W_alpha", "b_alpha"),
                (f"K{i}", f"S{i}", f"relw{i}", f"Wa{i}", f"ba{i}"))]))
        groups.append(("DistMult", [("rel_embedding:0", d["rel"])]))
        for g, ws in groups:
            grp = f.create_group(g)
            grp.attrs["weight_names"] = np.array([f"{g}/{w}".encode() for w, _ in ws])
            for w, a in ws:
                grp.create_dataset(f"{g}/{w}", data=a)
