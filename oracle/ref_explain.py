"""torch-CPU restatement of the reference explainers — TEST INFRASTRUCTURE ONLY (oracle/__init__.py).

References (all in /root/reference/explanation):
  explaiNE.get_pred + per-triple loop        explaiNE.py:12-32, 84-96
  computation graph                          GnnExplainer.py:13-24 (= IDDGCN_explain.py:16-27)
  GNNExplainer mask training                 GnnExplainer.py:26-74 (Keras Adam shared by all triples)
  IDDGCN explainer (+ structure loss)        IDDGCN_explain.py:30-118
  explanation metrics                        eval_test.py:15-39
Gradients w.r.t. adjacency values come from torch autograd of the reference formulation
(ref_model.layer_call's op order, with the SpMM A_r·E written as an index_add so the stored values
are leaves), float64 by default, independent of the HIP path's hand-derived backward + SDDMM.
"""
import numpy as np
import torch

from .ref_model import to_torch_params
from .ref_utils import get_adj_coo


def _spmm(rows, cols, vals, E):
    """A·E for the COO (rows, cols, vals): out[rows[k]] += vals[k] * E[cols[k]]."""
    return torch.zeros_like(E).index_add(0, rows, vals[:, None] * E[cols])


def _layer(E, hi, xh, ti, xt, ae, K, S, Wa, ba):
    """IDDGCN.py:60-79 with the relation aggregates AE_r precomputed (they do not depend on the
    layer input: every layer is fed all_e, IDDGCN.py:243/256/269)."""
    ho, to = xh @ S, xt @ S
    alpha = torch.softmax(xh @ Wa + ba, dim=-1)
    for i in range(K.shape[0]):
        w = torch.sigmoid(alpha[:, i])[:, None]
        ho = ho + w * (ae[i][hi] @ K[i])
        to = to + w * (ae[i][ti] @ K[i])
    return torch.sigmoid(ho), torch.sigmoid(to)


def forward_with_values(P, triples, coo, vals):
    """get_IDDGCN_Model forward (IDDGCN.py:226-275 + DistMult :103-109) on adjacency values `vals`
    (list of torch tensors, one per relation, in `coo` entry order)."""
    E = P["E"]
    tr = torch.as_tensor(np.asarray(triples), dtype=torch.int64)
    h, r, t = tr[:, 0], tr[:, 1], tr[:, 2]
    ae = [_spmm(torch.as_tensor(idx[:, 0]), torch.as_tensor(idx[:, 1]), v, E) for (idx, _), v in zip(coo, vals)]
    xh, xt = E[h], E[t]
    for l in (1, 2, 3):
        xh, xt = _layer(E, h, xh, t, xt, ae, P[f"K{l}"], P[f"S{l}"], P[f"Wa{l}"], P[f"ba{l}"])
    return torch.sigmoid(torch.sum(xh * P["rel"][r] * xt, dim=-1))


def value_grads(params, triple, coo, values=None, dtype=torch.float64):
    """(p, [d p / d values_r]) for one scored triple (explaiNE.py:85-94)."""
    P = to_torch_params(params, dtype, requires_grad=False)
    vals = [torch.tensor(np.asarray(v if values is None else values[i]), dtype=dtype, requires_grad=True)
            for i, (_, v) in enumerate(coo)]
    p = forward_with_values(P, np.asarray(triple)[None], coo, vals)[0]
    g = torch.autograd.grad(p, vals)
    return float(p.detach()), [x.numpy() for x in g]


def get_pred(coo, grads, top_k):
    """explaiNE.get_pred (explaiNE.py:12-32), literally: a python list of (idx, rel, score), sorted
    by score with reverse=True (stable), top_k, triples [head, rel, tail] from the indices."""
    scores = []
    for i, g in enumerate(grads):
        for idx, score in enumerate(g):
            scores.append((idx, i, score))
    top = sorted(scores, key=lambda x: x[2], reverse=True)[:top_k]
    trip = [[coo[rel][0][idx, 0], rel, coo[rel][0][idx, 1]] for idx, rel, _ in top]
    return np.array(trip, dtype=np.int64).reshape(-1, 3), np.array([s for _, _, s in top])


def explaine(params, adjacency_data, test_triples, N, R, top_k=10, dtype=torch.float64):
    coo = get_adj_coo(adjacency_data, N, R)
    out = [get_pred(coo, value_grads(params, tr, coo, dtype=dtype)[1], top_k) for tr in np.asarray(test_triples)]
    return np.stack([o[0] for o in out]), np.stack([o[1] for o in out])


def computation_graph(head, tail, data):
    """GnnExplainer.py:13-24."""
    data = np.asarray(data)
    nb = lambda n: np.concatenate([data[data[:, 0] == n], data[data[:, 2] == n]])  # noqa: E731
    return np.concatenate([nb(head), nb(tail)])


def mask_explainer(params, adjacency_data, test_triples, N, R, init_value, num_epochs=5, lr=1e-3, threshold=0.2,
                   target_ratios=None, top_k=10, dtype=torch.float64):
    """GnnExplainer.replica_step / IDDGCN_explain.wgnnexplainer_step with a Keras-Adam (ApplyAdam form,
    lr, b1=.9, b2=.999, eps=1e-7) shared across triples over dense (N, N) masks per relation.
    Returns (preds, scores, final masked values per triple)."""
    P = to_torch_params(params, dtype, requires_grad=False)
    init = np.asarray(init_value, np.float64).reshape(N, N)
    masks = [init.copy() for _ in range(R)]
    m = [np.zeros((N, N)) for _ in range(R)]
    v = [np.zeros((N, N)) for _ in range(R)]
    it = 0
    preds, scores, finals = [], [], []
    for tr in np.asarray(test_triples):
        coo = get_adj_coo(computation_graph(tr[0], tr[2], adjacency_data), N, R)
        base = [torch.as_tensor(np.asarray(val), dtype=dtype) for _, val in coo]
        before = forward_with_values(P, tr[None], coo, base)[0].detach()
        for _ in range(num_epochs):
            mk = [torch.tensor(masks[r], dtype=dtype, requires_grad=True) for r in range(R)]
            mv = [base[r] * torch.sigmoid(mk[r][coo[r][0][:, 0], coo[r][0][:, 1]]) for r in range(R)]
            pred = forward_with_values(P, tr[None], coo, mv)[0]
            loss = -before * torch.log(pred + 1e-5)
            if target_ratios is not None:
                counts = torch.stack([x.sum() for x in mv])
                ratios = counts / counts.sum()
                loss = (loss + torch.mean((torch.as_tensor(target_ratios, dtype=dtype) - ratios) ** 2)) / 2.0
            grads = torch.autograd.grad(loss, mk)
            it += 1
            b1, b2, eps = 0.9, 0.999, 1e-7
            alpha = lr * np.sqrt(1 - b2 ** it) / (1 - b1 ** it)
            for r in range(R):
                g = grads[r].numpy()
                m[r] = m[r] + (g - m[r]) * (1 - b1)
                v[r] = v[r] + (g * g - v[r]) * (1 - b2)
                masks[r] = masks[r] - alpha * m[r] / (np.sqrt(v[r]) + eps)
        mv = [np.asarray(coo[r][1], np.float64) * (1 / (1 + np.exp(-masks[r][coo[r][0][:, 0], coo[r][0][:, 1]])))
              for r in range(R)]
        trip, sc = [], []
        for r in range(R):
            keep = mv[r] > threshold
            kept = coo[r][0][keep]
            if kept.sum() == 0:
                continue
            trip.append(np.stack([kept[:, 0], np.full(len(kept), r), kept[:, 1]], 1))
            sc.append(mv[r][keep])
        trip = np.concatenate(trip) if trip else np.zeros((0, 3), np.int64)
        sc = np.concatenate(sc) if sc else np.zeros((0,))
        order = np.argsort(-sc, kind="stable")[:top_k]
        preds.append(trip[order])
        scores.append(sc[order])
        finals.append(np.concatenate(mv))
        masks = [init.copy() for _ in range(R)]
    return preds, scores, finals
