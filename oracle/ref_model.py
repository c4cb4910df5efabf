"""torch-CPU restatement of the IDDGCN model, loss and optimizer.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).  It follows the reference
op-for-op, in the *reference formulation* (per-edge GEMMs, ``A_r·E``
recomputed inside every layer call), so that:

  * gradients come from torch autograd of the reference op graph, independent
    of the hand-derived backward in the HIP path;
  * timing it on the host gives the "reference CPU path" baseline of bench.py.

References (all in /root/reference/prediction):
  IDDGCN_Layer.call         IDDGCN.py:60-79
  DistMult.call             IDDGCN.py:103-109
  model wiring              IDDGCN.py:201-285
  train_step (pos+neg, BCE, x 1/num_entities, Adam)  IDDGCN.py:123-178
  Keras 2.7 BinaryCrossentropy (from_logits=False, eps=1e-7 clip) and
  Keras 2.7 Adam (beta1=.9, beta2=.999, eps=1e-7) — third-party semantics of
  tensorflow==2.7.0 (README.md:17-19), restated from its published algorithm.
"""
import math

import numpy as np
import torch

LAYER_KEYS = ("relation_kernels", "self_kernel", "relation_weights", "W_alpha", "b_alpha")
EPS_BCE = 1e-7


def init_params(num_entities, num_relations, dim, seed=89, dtype=np.float32):
    """Reference-distribution initialisation (IDDGCN.py:25-58, 92-101, 221-224).

    TF's seeded initialisers cannot be replayed bit-for-bit, so this draws the
    same *distributions* from numpy: E~U[0,1), K,S~N(0,1), relation_weights
    ~U(-.05,.05), W_alpha glorot-uniform, b_alpha=0, rel~N(0,1).
    """
    rng = np.random.default_rng(seed)
    p = {"E": rng.random((num_entities, dim))}
    lim = math.sqrt(6.0 / (dim + num_relations))
    for l in (1, 2, 3):
        p[f"K{l}"] = rng.standard_normal((num_relations, dim, dim))
        p[f"S{l}"] = rng.standard_normal((dim, dim))
        p[f"relw{l}"] = rng.uniform(-0.05, 0.05, (num_relations,))
        p[f"Wa{l}"] = rng.uniform(-lim, lim, (dim, num_relations))
        p[f"ba{l}"] = np.zeros((num_relations,))
    p["rel"] = rng.standard_normal((num_relations, dim))
    return {k: v.astype(dtype) for k, v in p.items()}


def adj_to_torch(adj_coo, num_entities, dtype=torch.float64):
    """(indices, values) per relation -> torch sparse COO (N x N)."""
    mats = []
    for idx, val in adj_coo:
        i = torch.as_tensor(np.asarray(idx).T.copy(), dtype=torch.int64)
        v = torch.as_tensor(np.asarray(val), dtype=dtype)
        mats.append(torch.sparse_coo_tensor(i, v, (num_entities, num_entities)).coalesce())
    return mats


def layer_call(E, head_idx, head_e, tail_idx, tail_e, adj, K, S, Wa, ba, ae_cache=None):
    """IDDGCN.py:60-79, op for op.  ``ae_cache`` (a dict) keeps A_r·E across the calls of one forward:
    the reference recomputes it in every layer from the same E (:243,256,269), so the cached value is
    the identical tensor (a plain common-subexpression reuse for large-graph tests)."""
    head_output = head_e @ S                                     # :62
    tail_output = tail_e @ S                                     # :63
    alpha = torch.softmax(head_e @ Wa + ba, dim=-1)              # :66
    for i in range(K.shape[0]):                                  # :68
        if ae_cache is not None and i in ae_cache:
            sum_embeddings = ae_cache[i]
        else:
            sum_embeddings = torch.sparse.mm(adj[i], E)          # :69-70
            if ae_cache is not None:
                ae_cache[i] = sum_embeddings
        head_update = sum_embeddings[head_idx]                   # :71
        tail_update = sum_embeddings[tail_idx]                   # :72
        relation_weight = torch.sigmoid(alpha[:, i])             # :75
        head_output = head_output + relation_weight[:, None] * (head_update @ K[i])   # :76
        tail_output = tail_output + relation_weight[:, None] * (tail_update @ K[i])   # :77
    return torch.sigmoid(head_output), torch.sigmoid(tail_output)  # :79


def model_forward(P, heads, rels, tails, adj, return_layers=False, return_logits=False, ae_cache=None,
                  tail_round=None):
    """get_IDDGCN_Model wiring (IDDGCN.py:226-275) + DistMult (:103-109).  Returns the probabilities
    [, the per-layer (x_h, x_t) outputs] [, the pre-sigmoid DistMult logits (:108, inside the sigmoid)].
    ``tail_round`` (test hook, default None = the reference): applied to each layer's tail output x_t^l, to
    replay a storage rounding of the tail activations (the build's bf16-feature mode stores x^1..x^3 as
    bf16) so its kernels can be compared with float64 arithmetic on the same rounded tables."""
    E = P["E"]
    h = torch.as_tensor(heads, dtype=torch.int64)
    r = torch.as_tensor(rels, dtype=torch.int64)
    t = torch.as_tensor(tails, dtype=torch.int64)
    xh, xt = E[h], E[t]                                          # :226-235
    layers = []
    for l in (1, 2, 3):                                          # :238-274 (all_e = E feeds every layer)
        xh, xt = layer_call(E, h, xh, t, xt, adj, P[f"K{l}"], P[f"S{l}"], P[f"Wa{l}"], P[f"ba{l}"], ae_cache)
        if tail_round is not None:
            xt = tail_round(xt)
        layers.append((xh, xt))
    rel_e = P["rel"][r]                                          # :106
    logit = torch.sum(xh * rel_e * xt, dim=-1)                   # :108 (argument of the sigmoid)
    score = torch.sigmoid(logit)                                 # :108
    out = (score,) + ((layers,) if return_layers else ()) + ((logit,) if return_logits else ())
    return out if len(out) > 1 else score


def keras_bce(y_true, y_pred):
    """Keras 2.7 backend.binary_crossentropy (from_logits=False) + mean.

    The op feeding the loss is ConcatV2 (IDDGCN.py:161), so the logits fast
    path is not taken: output is clipped to [eps, 1-eps] and eps is added
    inside both logs.  Reduction SUM_OVER_BATCH_SIZE over a (1, T) input is
    the plain mean.
    """
    eps = torch.tensor(EPS_BCE, dtype=y_pred.dtype)
    out = torch.clamp(y_pred, eps, 1.0 - eps)
    bce = y_true * torch.log(out + eps) + (1.0 - y_true) * torch.log(1.0 - out + eps)
    return torch.mean(-bce)


def to_torch_params(params, dtype=torch.float64, requires_grad=True):
    return {k: torch.tensor(np.asarray(v), dtype=dtype, requires_grad=requires_grad and not k.startswith("relw"))
            for k, v in params.items()}


def train_step_grads(params, pos, neg, adj_coo, num_entities, dtype=torch.float64, scale_entities=None):
    """IDDGCN.py:123-178 up to tape.gradient.

    pos/neg are (B,3) int arrays of (head, rel, tail).  Returns
    (unscaled_loss, scores[pos..., neg...], grads dict).  ``relation_weights``
    receive no gradient (they are not used in IDDGCN_Layer.call).
    ``scale_entities`` (default ``num_entities``): the entity count of the loss
    scale ×1/num_entities (:168), for a problem relabelled onto a subset of a
    larger graph's entities (tests/fullsize_grads.py).
    """
    P = to_torch_params(params, dtype)
    adj = adj_to_torch(adj_coo, num_entities, dtype)
    pos = np.asarray(pos)
    neg = np.asarray(neg)
    y_pos = model_forward(P, pos[:, 0], pos[:, 1], pos[:, 2], adj)
    y_neg = model_forward(P, neg[:, 0], neg[:, 1], neg[:, 2], adj)
    y_pred = torch.cat([y_pos, y_neg])
    y_true = torch.cat([torch.ones_like(y_pos), torch.zeros_like(y_neg)])
    loss = keras_bce(y_true, y_pred)
    scaled = loss * (1.0 / (num_entities if scale_entities is None else scale_entities))   # :168
    keys = [k for k in P if P[k].requires_grad]
    grads = torch.autograd.grad(scaled, [P[k] for k in keys])
    return float(loss.detach()), y_pred.detach().numpy(), {k: g.numpy() for k, g in zip(keys, grads)}


class KerasAdam:
    """Keras 2.7 Adam (optimizer_v2/adam.py) with lr=1e-3, eps=1e-7.

    Dense variables follow TF's ApplyAdam kernel form
        m += (g - m)(1-b1); v += (g^2 - v)(1-b2); var -= alpha m / (sqrt(v)+eps)
    with alpha = lr sqrt(1-b2^t)/(1-b1^t).  Embedding-style variables whose
    gradient is IndexedSlices (entity_embeddings, DistMult rel_embedding) go
    through _resource_apply_sparse, which decays m/v densely and then adds the
    (deduplicated) slices — algebraically the same update in the form
        m = b1 m + (1-b1) g; v = b2 v + (1-b2) g^2.
    """

    SPARSE = ("E", "rel")

    def __init__(self, lr=1e-3, beta_1=0.9, beta_2=0.999, epsilon=1e-7):
        self.lr, self.b1, self.b2, self.eps = lr, beta_1, beta_2, epsilon
        self.m, self.v, self.iterations = {}, {}, 0

    def step(self, params, grads, dtype=np.float64):
        self.iterations += 1
        t = self.iterations
        f = dtype
        b1, b2, lr, eps = f(self.b1), f(self.b2), f(self.lr), f(self.eps)
        b1p, b2p = b1 ** f(t), b2 ** f(t)
        alpha = lr * np.sqrt(f(1) - b2p) / (f(1) - b1p)
        out = dict(params)
        for k, g in grads.items():
            g = np.asarray(g, dtype=f)
            m = self.m.setdefault(k, np.zeros_like(g))
            v = self.v.setdefault(k, np.zeros_like(g))
            if k in self.SPARSE:
                m = m * b1 + g * (f(1) - b1)
                v = v * b2 + (g * g) * (f(1) - b2)
            else:
                m = m + (g - m) * (f(1) - b1)
                v = v + (g * g - v) * (f(1) - b2)
            self.m[k], self.v[k] = m, v
            out[k] = (np.asarray(params[k], dtype=f) - alpha * m / (np.sqrt(v) + eps)).astype(f)
        return out


def predict(params, triples, adj_coo, num_entities, dtype=torch.float64, logits=False):
    """model.predict (IDDGCN_eval.py:97-105): forward only, returns the (B,) probabilities, or with
    ``logits=True`` (probabilities, pre-sigmoid DistMult scores)."""
    P = to_torch_params(params, dtype, requires_grad=False)
    adj = adj_to_torch(adj_coo, num_entities, dtype)
    tr = np.asarray(triples).astype(np.int64)
    with torch.no_grad():
        if logits:
            p, s = model_forward(P, tr[:, 0], tr[:, 1], tr[:, 2], adj, return_logits=True)
            return p.numpy(), s.numpy()
        return model_forward(P, tr[:, 0], tr[:, 1], tr[:, 2], adj).numpy()


def forward_detail(params, triples, adj_coo, num_entities, dtype=torch.float64, tail_round=None):
    """The forward of IDDGCN.py:226-275 on `triples` with everything a parity test compares: the
    probabilities, the pre-sigmoid DistMult logits and the per-layer outputs [(x_h^l, x_t^l)], l=1..3,
    as numpy arrays.  Cost O(len(triples)) plus one SpMM per relation per layer.  ``adj_coo`` may hold
    only the adjacency rows of the entities the triples touch (A_r·E is only gathered at h and t), which
    keeps the oracle cheap on million-node graphs.  ``tail_round``: see model_forward."""
    P = to_torch_params(params, dtype, requires_grad=False)
    adj = adj_to_torch(adj_coo, num_entities, dtype)
    tr = np.asarray(triples).astype(np.int64)
    with torch.no_grad():
        p, layers, s = model_forward(P, tr[:, 0], tr[:, 1], tr[:, 2], adj, return_layers=True, return_logits=True,
                                     ae_cache={}, tail_round=tail_round)
    return p.numpy(), s.numpy(), [(a.numpy(), b.numpy()) for a, b in layers]


def eval_metrics(y_true, y_prob, threshold=0.5):
    """IDDGCN_eval.py:106-122 metric block."""
    from sklearn.metrics import auc, confusion_matrix, precision_recall_curve, roc_auc_score
    y_pred = (np.asarray(y_prob) > threshold).astype(int)
    tn, fp, fn, tp = confusion_matrix(y_true, y_pred).ravel()
    prec, reca, _ = precision_recall_curve(np.array(y_true), np.array(y_prob))
    return {
        "tp": int(tp), "tn": int(tn), "fp": int(fp), "fn": int(fn),
        "accuracy": (tn + tp) / (tn + fp + fn + tp),
        "recall": tp / (tp + fn), "precision": tp / (tp + fp),
        "specificity": tn / (tn + fp),
        "f1": 2 * (tp / (tp + fp)) * (tp / (tp + fn)) / ((tp / (tp + fp)) + (tp / (tp + fn))),
        "roc_auc": roc_auc_score(y_true, y_prob),
        "aupr": auc(reca, prec),
    }
