"""Weight files: the repo's .npz layout and Keras h5 (h5py when importable, else iddgcn_amd/h5lite.py).

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


def _dec(s):
    return s.decode() if isinstance(s, bytes) else str(s)


def load_h5(path):
    """Keras ``load_weights`` of an .h5 file: the weighted layers in ``layer_names`` order, each
    layer's arrays in its ``weight_names`` order.  Uses h5py when importable, else the built-in
    reader (iddgcn_amd/h5lite.py)."""
    try:
        import h5py
    except ImportError:
        h5py = None
    weighted = []
    if h5py is not None:
        with h5py.File(path, "r") as f:
            for n in (_dec(x) for x in f.attrs["layer_names"]):
                wn = [_dec(w) for w in f[n].attrs["weight_names"]]
                if wn:
                    weighted.append([np.asarray(f[n][w], dtype=np.float32) for w in wn])
    else:
        from .h5lite import open_file
        f = open_file(path)
        for n in (_dec(x) for x in f.attrs["layer_names"]):
            wn = [_dec(w) for w in np.atleast_1d(f[n].attrs.get("weight_names", []))]
            if wn:
                weighted.append([np.asarray(f[n][w], dtype=np.float32) for w in wn])
    if len(weighted) != 5:
        raise ValueError(f"{path}: expected 5 weighted layers, found {len(weighted)}")
    out = {"E": weighted[0][0], "rel": weighted[4][0]}
    for l in (1, 2, 3):
        for k, a in zip(("K", "S", "relw", "Wa", "ba"), weighted[l]):
            out[f"{k}{l}"] = a
    return out


def keras_layout(model):
    """[(layer name, [(weight name, array), ...]), ...] as Keras save_weights lays the model out
    (IDDGCN.py:181-199): entity_embeddings, the three graph layers, DistMult."""
    d = model._named()
    groups = [("entity_embeddings", [("entity_embeddings/embeddings:0", d["E"])])]
    for i, l in enumerate(model.gcn_layers, 1):
        groups.append((l.name, [(f"{w}:0", d[k]) for w, k in zip(
            ("relation_kernels", "self_kernel", "relation_weights", "W_alpha", "b_alpha"),
            (f"K{i}", f"S{i}", f"relw{i}", f"Wa{i}", f"ba{i}"))]))
    groups.append(("DistMult", [("DistMult/rel_embedding:0", d["rel"])]))
    return groups


def save_h5(path, model):
    """Keras-h5 weight file (root attrs layer_names / backend / keras_version, one group per layer
    with a weight_names attribute, the arrays under their weight-name paths).  h5py when
    importable, else the built-in writer."""
    groups = keras_layout(model)
    names = [g for g, _ in groups]
    try:
        import h5py
    except ImportError:
        h5py = None
    if h5py is not None:
        with h5py.File(path, "w") as f:
            f.attrs["layer_names"] = np.array([n.encode() for n in names])
            f.attrs["backend"] = b"tensorflow"
            f.attrs["keras_version"] = b"2.7.0"
            for g, ws in groups:
                grp = f.create_group(g)
                grp.attrs["weight_names"] = np.array([w.encode() for w, _ in ws])
                for w, a in ws:
                    grp.create_dataset(w, data=a)
        return
    from .h5lite import write_file
    tree = {}
    for g, ws in groups:
        sub = {}
        for w, a in ws:
            node = sub
            parts = w.split("/")
            for part in parts[:-1]:
                node = node.setdefault(part, {})
            node[parts[-1]] = np.asarray(a, dtype=np.float32)
        tree[g] = (sub, {"weight_names": np.array([w.encode() for w, _ in ws])})
    write_file(path, tree, {"layer_names": np.array([n.encode() for n in names]), "backend": np.bytes_(b"tensorflow"),
                            "keras_version": np.bytes_(b"2.7.0")})
