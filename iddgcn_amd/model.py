"""Keras-shaped drop-in surface of the reference model (prediction/IDDGCN.py).

Names, constructor arguments, weight order and the fit/predict calling
convention follow the reference so that ``IDDGCN.py``'s ``__main__`` and
``IDDGCN_eval.py`` keep their shape:

    model = get_IDDGCN_Model(num_entities, num_relations, embedding_dim,
                             output_dim, seed, all_feature_matrix, mode, fold)
    model.compile(loss=BinaryCrossentropy(), optimizer=Adam(learning_rate=1e-3))
    model.fit(x=[ALL_INDICES, X[:, :, 0], X[:, :, 1], X[:, :, 2], ADJ_MATS],
              y=np.ones((1, B)), epochs=5000, batch_size=100, callbacks=[...])
    preds = model.predict(x=[ALL_INDICES, h, r, t, ADJ_MATS])      # (1, B)

Everything numeric runs in libiddgcn_hip.so on the GPU (engine.py); this
module only holds weights and wiring.  There is no CPU fallback.
"""
import math
import os

import numpy as np
import torch

from . import _lib as L
from . import ops
from .engine import NUM_LAYERS, Engine, FlatParams, GraphedTrainStep, KerasAdam
from .graph import DeviceAdjacency, SparseAdj, get_adj_mats  # noqa: F401  (re-export)
from .parallel import BucketedAllReduce, shard_triples, world

LAYER_WEIGHT_NAMES = ("relation_kernels", "self_kernel", "relation_weights", "W_alpha", "b_alpha")


# ---------------------------------------------------------------------------
# compile() arguments
# ---------------------------------------------------------------------------
class BinaryCrossentropy:
    """tf.keras.losses.BinaryCrossentropy() (from_logits=False), as used at IDDGCN.py:391."""

    def __init__(self, from_logits=False):
        if from_logits:
            raise NotImplementedError("the reference uses from_logits=False")


class Adam:
    """tf.keras.optimizers.Adam (IDDGCN.py:392): lr 1e-3, beta 0.9/0.999, eps 1e-7."""

    def __init__(self, learning_rate=0.001, beta_1=0.9, beta_2=0.999, epsilon=1e-7):
        self.learning_rate, self.beta_1, self.beta_2, self.epsilon = learning_rate, beta_1, beta_2, epsilon


class Callback:
    """Minimal keras.callbacks.Callback."""

    def set_model(self, model):
        self.model = model

    def on_epoch_end(self, epoch, logs=None):
        pass


class History(Callback):
    def __init__(self):
        self.history = {}
        self.epoch = []

    def on_epoch_end(self, epoch, logs=None):
        self.epoch.append(epoch)
        for k, v in (logs or {}).items():
            self.history.setdefault(k, []).append(v)


class SaveWeightsCallback(Callback):
    """IDDGCN.py:181-199: save the model weights at the listed epochs."""

    def __init__(self, save_epochs, save_path_template, mode, fold, learning_rate, batch_size, EMBEDDING_DIM):
        self.save_epochs = save_epochs
        self.save_path_template = save_path_template
        self.mode, self.fold = mode, fold
        self.learning_rate, self.batch_size, self.EMBEDDING_DIM = learning_rate, batch_size, EMBEDDING_DIM

    def on_epoch_end(self, epoch, logs=None):
        if epoch + 1 in self.save_epochs:
            filename = self.save_path_template.format(mode=self.mode, fold=self.fold, epoch=epoch + 1,
                                                      learning_rate=self.learning_rate, batch_size=self.batch_size,
                                                      EMBEDDING_DIM=self.EMBEDDING_DIM)
            self.model.save_weights(filename)
            print(f"\nSaved weights for epoch {epoch + 1} to {filename}")


# ---------------------------------------------------------------------------
# layers (weight holders with the reference's shapes, order and initialisers)
# ---------------------------------------------------------------------------
def _glorot_uniform(rng, shape):
    lim = math.sqrt(6.0 / (shape[0] + shape[1]))
    return rng.uniform(-lim, lim, shape)


# Initialisation schemes.
#   "tf27" (default): TensorFlow 2.7 / Keras 2.7's own draws, replayed (iddgcn_amd/tf_random.py): after
#       tf.random.set_seed(seed) (IDDGCN.py:292) the seeded initialisers (RandomUniform / RandomNormal with
#       seed=SEED) are stateful Philox ops keyed (SEED, SEED) whose cached kernel continues its stream from call to
#       call, and the unseeded ones ('uniform' relation_weights, glorot_uniform W_alpha) take op seeds from the
#       eager context's Random(SEED).  Bit for bit the reference's initial relation_weights (all 5 bundled folds)
#       and the untouched entity rows (folds 0, 1, 4); the Box-Muller normals go through the host libm as TF's
#       CPU kernel does (their bits are not pinned by any reference file: every normal-initialised weight is
#       trained).  A model replays a fresh process's draws; ``tf_models_before`` / ``tf_extra_op_seeds`` place
#       it later in a process (the bundled fold 3: 1 and 1).
#   "independent": every weight an independent numpy draw of the same distribution (round 1).
INIT_SCHEMES = ("tf27", "independent")


def _session(seed, tf_random):
    """The TFRandom state a weight is drawn from: the model's shared one, or a fresh set_seed(seed) state."""
    if tf_random is not None:
        return tf_random
    from .tf_random import TFRandom
    return TFRandom(seed)


class Layer:
    def __init__(self, name):
        self.name = name

    def get_weights(self):
        return [w.copy() for w in self._weights]

    def set_weights(self, ws):
        if len(ws) != len(self._weights):
            raise ValueError(f"{self.name}: expected {len(self._weights)} arrays, got {len(ws)}")
        for i, (old, new) in enumerate(zip(self._weights, ws)):
            new = np.asarray(new, dtype=np.float32)
            if new.shape != old.shape:
                raise ValueError(f"{self.name}: weight {i} shape {new.shape} != {old.shape}")
            self._weights[i] = new.copy()


class Embedding(Layer):
    """Keras Embedding(input_dim=N, output_dim=D), RandomUniform(0, 1) init (IDDGCN.py:215-225)."""

    def __init__(self, input_dim, output_dim, seed=None, name="entity_embeddings", init="tf27", tf_random=None):
        super().__init__(name)
        if init == "tf27" and seed is not None:
            w = _session(seed, tf_random).uniform((input_dim, output_dim), 0, 1, seed=int(seed))
        else:
            w = np.random.default_rng(seed).random((input_dim, output_dim))
        self._weights = [w.astype(np.float32)]


class IDDGCN_Layer(Layer):
    """IDDGCN.py:16-79.  Weights in the reference's order:
    [relation_kernels (R,D,D), self_kernel (D,D), relation_weights (R,), W_alpha (D,R), b_alpha (R,)].
    ``relation_weights`` is created (it occupies a slot of the h5 layout) but,
    as in the reference, never used by ``call`` and never trained."""

    def __init__(self, num_entities, num_relations, output_dim, seed, name="iddgcn__layer", init="tf27",
                 layer_index=0, tf_random=None, **kwargs):
        super().__init__(kwargs.get("name", name))
        self.num_entities, self.num_relations, self.output_dim, self.seed = (num_entities, num_relations,
                                                                             output_dim, seed)
        if init not in INIT_SCHEMES:
            raise ValueError(f"init must be one of {INIT_SCHEMES}")
        R, D = num_relations, output_dim
        if init == "tf27":
            tf = _session(seed, tf_random)
            K = tf.normal((R, D, D), 0.0, 1.0, seed=int(seed))      # RandomNormal(0, 1, seed) (:25-30)
            S = tf.normal((D, D), 0.0, 1.0, seed=int(seed))         # the same kernel, its stream continued (:31-36)
            relw = tf.uniform((R,), -0.05, 0.05)                    # 'uniform' (:39-44), an op seed
            Wa = tf.glorot_uniform((D, R))                          # glorot_uniform (:47-52), an op seed
        else:
            rng = np.random.default_rng(seed)
            K = rng.standard_normal((R, D, D))
            S = rng.standard_normal((D, D))
            relw = rng.uniform(-0.05, 0.05, (R,))
            Wa = _glorot_uniform(rng, (D, R))
        self._weights = [K.astype(np.float32), S.astype(np.float32), relw.astype(np.float32), Wa.astype(np.float32),
                         np.zeros((R,), np.float32)]

    def __call__(self, inputs, weights=None):
        """IDDGCN.py:60-79 on GPU tensors: inputs = [embeddings (N,D), head_idx (B,), head_e (B,D),
        tail_idx (B,), tail_e (B,D), adj_mats].  Returns (sigmoid(head_out), sigmoid(tail_out)), each (B, D),
        differentiable (autograd.IDDGCNLayerFunction) w.r.t. embeddings, head_e, tail_e and — passed as
        ``weights=[relation_kernels, self_kernel, W_alpha, b_alpha]`` tensors — the layer weights (the
        layer's own weights are used as constants otherwise)."""
        from .autograd import IDDGCNLayerFunction
        embeddings, head_idx, head_e, tail_idx, tail_e, *adj = inputs
        adj = _unwrap_adj(adj)
        dev = embeddings.device
        N, D, R = self.num_entities, self.output_dim, self.num_relations
        if weights is None:
            K, S, _, Wa, ba = [torch.as_tensor(w, device=dev) for w in self._weights]
        else:
            K, S, Wa, ba = weights
        dadj = adj if isinstance(adj, DeviceAdjacency) else DeviceAdjacency(adj, N, dev)
        B = head_e.shape[0]
        hi = head_idx.to(device=dev, dtype=torch.int32).contiguous()
        ti = tail_idx.to(device=dev, dtype=torch.int32).contiguous()
        if B and (int(hi.min()) < 0 or int(hi.max()) >= N or int(ti.min()) < 0 or int(ti.max()) >= N):
            raise L.IddgcnError("head/tail index out of range")
        if tuple(embeddings.shape) != (N, D) or tuple(head_e.shape) != (B, D) or tuple(tail_e.shape) != (B, D):
            raise L.IddgcnError("embeddings (N, D), head_e and tail_e (B, D) expected")
        return IDDGCNLayerFunction.apply(embeddings, head_e, tail_e, K, S, Wa, ba, hi, ti, dadj)


class DistMult(Layer):
    """IDDGCN.py:82-109: rel_embedding (R, D) ~ N(0,1); score = sigmoid(sum h*r*t), shape (1, B)."""

    def __init__(self, num_relations, seed, name="DistMult", embedding_dim=None, init="tf27", tf_random=None,
                 **kwargs):
        super().__init__(name)
        self.num_relations, self.seed, self.init = num_relations, seed, init
        self._tf = tf_random
        self._weights = []
        if embedding_dim is not None:
            self.build(embedding_dim)

    def build(self, embedding_dim):
        R, D = self.num_relations, embedding_dim
        if self.init == "tf27":           # RandomNormal(0, 1, seed) (:90-99): the layers' normal kernel, continued
            w = _session(self.seed, self._tf).normal((R, D), 0.0, 1.0, seed=int(self.seed))
        else:
            w = np.random.default_rng(self.seed).standard_normal((R, D))
        self._weights = [w.astype(np.float32)]

    def __call__(self, inputs, logits=False, rel_embedding=None):
        """sigmoid(sum head_e * rel[rel_idx] * tail_e) as (1, B), differentiable (autograd.DistMultFunction)
        w.r.t. head_e, tail_e and a ``rel_embedding`` tensor if given; ``logits=True``: the sum itself."""
        from .autograd import DistMultFunction
        head_e, rel_idx, tail_e = inputs
        dev = head_e.device
        if not self._weights:
            self.build(head_e.shape[-1])
        rel = torch.as_tensor(self._weights[0], device=dev) if rel_embedding is None else rel_embedding
        B = head_e.shape[0]
        ri = rel_idx.to(device=dev, dtype=torch.int32).contiguous()
        if B and (int(ri.min()) < 0 or int(ri.max()) >= self.num_relations):
            raise L.IddgcnError("relation index out of range")
        if logits:
            ident = torch.arange(B, device=dev, dtype=torch.int32)
            p, s = torch.empty(B, device=dev), torch.empty(B, device=dev)
            ops.distmult_bce(head_e.contiguous(), ident, tail_e.contiguous(), ri, rel.contiguous(), p_out=p, s_out=s)
            return s.view(1, B)
        return DistMultFunction.apply(head_e, rel, tail_e, ri).view(1, B)


# ---------------------------------------------------------------------------
# model
# ---------------------------------------------------------------------------
def _unwrap_adj(adj):
    """The trailing inputs after (all, h, r, t) or (E, h, h_e, t, t_e): one DeviceAdjacency, one
    nested list/tuple of sparse matrices, or the matrices spliced in."""
    if len(adj) == 1 and isinstance(adj[0], (list, tuple, DeviceAdjacency)):
        return adj[0]
    return adj


def _squeeze_idx(a):
    if isinstance(a, torch.Tensor):
        a = a.cpu().numpy()
    a = np.asarray(a)
    return (a[0] if a.ndim == 2 else a).astype(np.int64)


class IDDGCN_Model:
    """IDDGCN.py:112-178 (custom train_step) + get_IDDGCN_Model wiring (:201-285)."""

    def __init__(self, num_entities, num_relations, embedding_dim, output_dim, seed, mode=0, fold=0,
                 neg_weight=1.0, init="tf27", tf_models_before=0, tf_extra_op_seeds=0):
        if embedding_dim != output_dim:
            raise ValueError("embedding_dim must equal output_dim (IDDGCN.py:307-308)")
        self.num_entities, self.num_relations, self.dim = num_entities, num_relations, embedding_dim
        self.seed, self.mode, self.fold, self.neg_weight = seed, mode, fold, neg_weight
        if init not in INIT_SCHEMES:
            raise ValueError(f"init must be one of {INIT_SCHEMES}")
        tf = None
        if init == "tf27":      # one eager random state for the whole model, drawn in the reference's order
            from .tf_random import TFRandom, draw_model
            tf = TFRandom(seed)
            for _ in range(tf_models_before):
                draw_model(tf, num_entities, num_relations, embedding_dim, seed)
            for _ in range(tf_extra_op_seeds):
                tf.get_seed()
        self.entity_embeddings = Embedding(num_entities, embedding_dim, seed, init=init, tf_random=tf)
        self.gcn_layers = [IDDGCN_Layer(num_entities, num_relations, output_dim, seed, init=init, layer_index=i,
                                        tf_random=tf, name="iddgcn__layer" + ("" if i == 0 else f"_{i}"))
                           for i in range(3)]
        self.distmult = DistMult(num_relations, seed, embedding_dim=embedding_dim, init=init, tf_random=tf)
        self.layers = [self.entity_embeddings, *self.gcn_layers, self.distmult]
        self.neg_triples = None         # set to override the reference's .npy negatives
        self.neg_path_template = "../datasets/prediction_datasets/mode{mode}_fold{fold}_X_train_neg.npy"
        self.optimizer = None
        self.stop_training = False
        self._engine = None
        self._dev = None
        self._opt_state = None
        self._graph_cache = {}
        # fit(): after one eager epoch, replay the captured step (HIP graph) for the rest
        self.use_graph = True

    # -- Keras-ish plumbing ----------------------------------------------------
    def get_layer(self, name):
        for l in self.layers:
            if l.name == name:
                return l
        raise ValueError(f"No such layer: {name}")

    @property
    def weights(self):
        return [w for l in self.layers for w in l.get_weights()]

    def get_weights(self):
        return self.weights

    def set_weights(self, ws):
        i = 0
        for l in self.layers:
            n = len(l._weights)
            l.set_weights(ws[i:i + n])
            i += n
        self._invalidate()

    def compile(self, loss=None, optimizer=None, **kwargs):
        if loss is not None and not isinstance(loss, BinaryCrossentropy) and loss not in ("binary_crossentropy",):
            raise NotImplementedError("IDDGCN trains with Keras BinaryCrossentropy (IDDGCN.py:391)")
        self.optimizer = optimizer if optimizer is not None else Adam()
        self._opt_state = None

    def reset_states(self):
        pass

    # -- weights <-> device ------------------------------------------------------
    def _named(self):
        d = {"E": self.entity_embeddings._weights[0], "rel": self.distmult._weights[0]}
        for i, l in enumerate(self.gcn_layers, 1):
            K, S, relw, Wa, ba = l._weights
            d.update({f"K{i}": K, f"S{i}": S, f"relw{i}": relw, f"Wa{i}": Wa, f"ba{i}": ba})
        return d

    def _set_named(self, d):
        self.entity_embeddings._weights[0] = np.asarray(d["E"], np.float32).copy()
        self.distmult._weights = [np.asarray(d["rel"], np.float32).copy()]
        for i, l in enumerate(self.gcn_layers, 1):
            l._weights = [np.asarray(d[k], np.float32).copy() for k in
                          (f"K{i}", f"S{i}", f"relw{i}", f"Wa{i}", f"ba{i}")]

    def _device_state(self):
        if self._engine is None:
            self._dev = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else None
            if self._dev is None:
                raise L.IddgcnError("IDDGCN_Model needs a GPU (no CPU fallback)")
            self._engine = Engine(self.num_entities, self.num_relations, self.dim, self._dev)
            self._params = FlatParams(self.num_entities, self.num_relations, self.dim, self._dev)
            self._grads = FlatParams(self.num_entities, self.num_relations, self.dim, self._dev)
            self._params.load(self._named())
        return self._engine

    def _sync_to_host(self):
        if self._engine is not None:
            d = self._named()
            d.update(self._params.to_numpy())
            self._set_named(d)

    def _invalidate(self):
        if self._engine is not None:
            self._params.load(self._named())

    def _adjacency(self, adj_mats):
        if isinstance(adj_mats, DeviceAdjacency):       # get_adj_mats(..., device=cuda)
            return adj_mats
        # key on the caller's objects (the list itself, or the tuple of its relation matrices when the
        # list was spliced into x): rebuilt only when the caller hands over a different graph
        key = tuple(id(a) for a in adj_mats)
        hit = self._graph_cache.get(key)
        if hit is not None and all(a is b for a, b in zip(hit[0], adj_mats)):
            return hit[1]
        dadj = DeviceAdjacency(list(adj_mats), self.num_entities, self._dev)
        self._graph_cache = {key: (list(adj_mats), dadj)}
        return dadj

    def save_weights(self, filepath):
        """Keras-h5 for a ``.h5`` path (IDDGCN.py:181-199; h5py or the built-in writer), else .npz."""
        self._sync_to_host()
        d = self._named()
        os.makedirs(os.path.dirname(os.path.abspath(filepath)), exist_ok=True)
        if filepath.endswith(".h5"):
            from .weights_io import save_h5
            save_h5(filepath, self)
        else:
            np.savez(filepath, **d)

    def load_weights(self, filepath):
        from .weights_io import load_any
        self._set_named(load_any(filepath, self))
        self._invalidate()

    # -- calls ---------------------------------------------------------------
    def _unpack(self, x):
        """x = [ALL_INDICES, h, r, t, ADJ_MATS] (IDDGCN.py:399-407).  ADJ_MATS may be the reference's
        list of per-relation sparse matrices, spliced in or nested, or one DeviceAdjacency
        (get_adj_mats(..., device=cuda)).  The adjacency object is returned as the caller passed it, so
        the graph cache (keyed on it) hits across fit/predict calls."""
        all_idx, h, r, t, *adj = x
        adj = _unwrap_adj(adj)
        return _squeeze_idx(h), _squeeze_idx(r), _squeeze_idx(t), adj

    def predict(self, x, batch_size=None, verbose=0, **kwargs):
        """model.predict (IDDGCN_eval.py:61-69,97-105): returns (1, B) probabilities."""
        eng = self._device_state()
        h, r, t, adj = self._unpack(x)
        dadj = self._adjacency(adj)
        ed = eng.edges(np.stack([h, r, t], 1))
        p = eng.predict(self._params, dadj, ed)
        return p.detach().cpu().numpy().reshape(1, -1)

    def predict_logits(self, x):
        """The pre-sigmoid DistMult scores of model.predict's edges, (1, B): the argument of the sigmoid
        at IDDGCN.py:108 (what the reference's y_pred is the sigmoid of)."""
        eng = self._device_state()
        h, r, t, adj = self._unpack(x)
        dadj = self._adjacency(adj)
        ed = eng.edges(np.stack([h, r, t], 1))
        _, s = eng.predict(self._params, dadj, ed, logits=True)
        return s.detach().cpu().numpy().reshape(1, -1)

    def __call__(self, x, training=False):
        return torch.as_tensor(self.predict(x))

    def _negatives(self):
        if self.neg_triples is not None:
            neg = np.asarray(self.neg_triples)
        else:
            neg = np.load(self.neg_path_template.format(mode=self.mode, fold=self.fold))
        neg = neg[0] if neg.ndim == 3 else neg
        return neg.astype(np.int64)

    def fit(self, x=None, y=None, epochs=1, batch_size=None, verbose=1, callbacks=None, **kwargs):
        """Full-batch training (IDDGCN.py:399-412): each epoch is ONE train_step
        over all positives (x) and the negatives of the .npy file (IDDGCN.py:128-160).
        ``batch_size`` has no effect, exactly as in the reference (leading dim 1).
        Under torch.distributed the scored edges are sharded over ranks."""
        eng = self._device_state()
        if self.optimizer is None:
            self.compile()
        h, r, t, adj = self._unpack(x)
        pos = np.stack([h, r, t], 1)
        neg = self._negatives()
        triples = np.concatenate([pos, neg])
        labels = np.concatenate([np.ones(len(pos), np.float32), np.zeros(len(neg), np.float32)])
        rank, ws = world()
        my_tr, my_lab = shard_triples(triples, labels, rank, ws)
        dadj = self._adjacency(adj)
        ed = eng.edges(my_tr, my_lab)
        if self._opt_state is None:
            o = self.optimizer
            self._opt_state = KerasAdam(self._params, o.learning_rate, o.beta_1, o.beta_2, o.epsilon)
        comm = BucketedAllReduce() if ws > 1 else None
        history = History()
        cbs = [history] + list(callbacks or [])
        for cb in cbs:
            cb.set_model(self)
        T = len(triples)
        graphed = None
        # per-epoch host work only when someone looks at it: else the replays run back to back and
        # the losses are read once at the end
        lazy = not verbose and all(isinstance(cb, History) for cb in cbs)
        pending = []
        for epoch in range(epochs):
            if graphed is None and self.use_graph and ws == 1 and epoch >= 1 and epochs - epoch > 1:
                graphed = GraphedTrainStep(eng, self._params, self._grads, self._opt_state, dadj, ed,
                                           epochs - epoch, t_global=T)
            if graphed is not None:
                loss_sum = graphed.replay()
            else:
                loss_sum = eng.train_step(self._params, self._grads, self._opt_state, dadj, ed, t_global=T,
                                          comm=comm)
            if lazy:
                pending.append(loss_sum if graphed is not None else loss_sum.clone())
                continue
            loss = float(loss_sum.item()) / T
            if verbose and rank == 0:
                print(f"Epoch {epoch + 1}/{epochs} - loss: {loss:.6f}")
            logs = {"loss": loss}
            if any(isinstance(cb, SaveWeightsCallback) and epoch + 1 in cb.save_epochs for cb in cbs):
                self._sync_to_host()
            for cb in cbs:
                cb.on_epoch_end(epoch, logs)
            if self.stop_training:
                break
        if pending:
            for epoch, l in enumerate(torch.cat([x.reshape(1) for x in pending]).cpu().tolist()):
                history.on_epoch_end(epoch, {"loss": l / T})
        self._sync_to_host()
        return history

    def train_step(self, data):
        """IDDGCN.py:123-178 for data = ([all, h, r, t, adj], y): one step, returns {'loss': ...}."""
        x, _ = data
        return {"loss": self.fit(x, None, epochs=1, verbose=0).history["loss"][0]}


def get_IDDGCN_Model(num_entities, num_relations, embedding_dim, output_dim, seed, all_feature_matrix=None, mode=0,
                     fold=0, init="tf27", **init_kw):
    """IDDGCN.py:201-285.  ``all_feature_matrix`` is accepted and unused, as in the
    reference (the Embedding's ``weights=`` argument is commented out, :219)."""
    return IDDGCN_Model(num_entities, num_relations, embedding_dim, output_dim, seed, mode=mode, fold=fold, init=init,
                        **init_kw)
