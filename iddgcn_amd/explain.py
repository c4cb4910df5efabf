"""Explainers on the MI355X path: the reference's three link-prediction
explainers, driven by the same HIP engine as training.

* explaiNE (explanation/explaiNE.py): for each test triple, the gradient of the predicted
  probability w.r.t. every adjacency VALUE (``tape.gradient(pred, adj_mat.values)``,
  explaiNE.py:85-94), ranked, top-k (``get_pred``, explaiNE.py:12-32).
* GNNExplainer (explanation/GnnExplainer.py) and the IDDGCN explainer
  (explanation/IDDGCN_explain.py): per test triple, the computation graph (edges touching the
  head or the tail, GnnExplainer.py:13-24) is masked as ``adj * sigmoid(mask)``; the masks are
  trained for a few epochs with Keras Adam on ``-before_pred * log(pred + 1e-5)`` (plus, for the
  IDDGCN explainer, a relation-ratio structure loss, IDDGCN_explain.py:30-41), then the masked
  values above a threshold are ranked.

All three need one primitive on the hot path: the gradient of the prediction w.r.t. the adjacency
values.  ``Engine.value_grads`` gets it from one forward + backward with the prediction seed and
one SDDMM (``iddgcn_sddmm_csr_f32``); masked values go to the device CSR with
``DeviceAdjacency.set_values`` (no rebuild).  Reference semantics kept on purpose:
* the Adam optimizer of the mask explainers is created ONCE and shared by all test triples (its
  iterations and moment slots carry over; the masks are reset to ``init_value`` after each triple,
  GnnExplainer.py:72-73), and it is the dense-variable form (ApplyAdam) over the full (N, N) mask
  of every relation;
* ranking is stable descending (Python ``sorted(..., reverse=True)`` in get_pred).
TF's seeded ``tf.random.normal`` mask init cannot be replayed without TF: pass ``init_value`` to
use a specific one (default: numpy N(0,1) with the given seed).
"""
import numpy as np
import torch

from . import ops
from ._lib import IddgcnError
from .graph import DeviceAdjacency, _as_triples, get_adj_mats


# -- host helpers (pure numpy) ---------------------------------------------------------------
def get_neighbors(data, node_idx):
    """GnnExplainer.py:13-17: triples with head == node, then triples with tail == node."""
    data = _as_triples(data)
    return np.concatenate([data[data[:, 0] == node_idx], data[data[:, 2] == node_idx]], 0)


def get_computation_graph(head, rel, tail, data):
    """GnnExplainer.py:19-24 / IDDGCN_explain.py:21-27 (duplicates kept; get_adj_mats dedups)."""
    return np.concatenate([get_neighbors(data, head), get_neighbors(data, tail)], 0)


def get_pred(adj_mats, value_grads, top_k):
    """explaiNE.get_pred (explaiNE.py:12-32) on per-relation value gradients (numpy arrays).

    Scores are visited relation by relation in entry order and ranked by a stable descending sort;
    returns ([top_k, 3] triples (head, rel, tail), [top_k] scores)."""
    rels = np.concatenate([np.full(len(g), r, np.int64) for r, g in enumerate(value_grads)])
    idx = np.concatenate([np.arange(len(g), dtype=np.int64) for g in value_grads])
    score = np.concatenate([np.asarray(g, np.float32) for g in value_grads])
    order = np.argsort(-score, kind="stable")[:top_k]
    triples = np.array([[adj_mats[rels[k]].indices[idx[k], 1], rels[k], adj_mats[rels[k]].indices[idx[k], 2]]
                        for k in order], dtype=np.int64).reshape(-1, 3)
    return triples, score[order]


def _model_state(model):
    eng = model._device_state()
    return eng, model._params


# -- explaiNE -------------------------------------------------------------------------------
def explaine(model, adjacency_data, test_triples, top_k=10, graph=True):
    """explaiNE.py __main__ loop (lines 57-101) for one fold: ADJACENCY_DATA = train ∪ test, one
    prediction-gradient per test triple.  Returns (preds [n, top_k, 3], scores [n, top_k]).

    graph=True (default): the per-triple work — the single-edge layout, forward + backward with the
    prediction seed, SDDMM, and the stable descending ranking (torch.sort on the device) — is
    captured once in a HIP graph and replayed per triple with no host round trip; graph=False runs
    the same launches eagerly and ranks on the host (get_pred)."""
    eng, params = _model_state(model)
    N, R = model.num_entities, model.num_relations
    adj_mats = get_adj_mats(adjacency_data, N, R)
    dadj = DeviceAdjacency(adj_mats, N, eng.device)
    triples = _as_triples(test_triples)
    if not graph:
        preds, scores = [], []
        for tr in triples:
            dv, _ = eng.value_grads(params, dadj, eng.edges(tr[None]))
            p, s = get_pred(adj_mats, [g.cpu().numpy() for g in dv], top_k)
            preds.append(p)
            scores.append(s)
        return np.stack(preds), np.stack(scores)
    return _ExplaineGraph(eng, params, dadj, top_k).run(triples)


class _SingleEdge:
    """A one-triple ScoredEdges whose device arrays are rewritten in place from a device (3,) int64
    triple (so a captured graph can be replayed for any triple)."""

    def __init__(self, eng, triple_buf):
        self.T, self.y = 1, None
        dev = eng.device
        self._tr = triple_buf
        self._ar = torch.arange(eng.N + 1, device=dev)
        self.h = torch.zeros(1, dtype=torch.int32, device=dev)
        self.r = torch.zeros(1, dtype=torch.int32, device=dev)
        self.t = torch.zeros(1, dtype=torch.int32, device=dev)
        self.tptr = torch.zeros(eng.N + 1, dtype=torch.int32, device=dev)
        self.hptr = torch.zeros(eng.N + 1, dtype=torch.int32, device=dev)
        self.hperm = torch.zeros(1, dtype=torch.int32, device=dev)
        self.inv = torch.zeros(1, dtype=torch.int64, device=dev)

    def refresh(self):
        """Device-side layout of the single edge (ScoredEdges semantics, graph-capturable)."""
        self.h.copy_(self._tr[0:1])
        self.r.copy_(self._tr[1:2])
        self.t.copy_(self._tr[2:3])
        self.tptr.copy_(self._ar > self._tr[2])      # segment of tail t is [tptr[t], tptr[t+1]) = [0, 1)
        self.hptr.copy_(self._ar > self._tr[0])

    def unsort(self, x):
        return x


class _ExplaineGraph:
    def __init__(self, eng, params, dadj, top_k):
        dev = eng.device
        self.k = min(top_k, dadj.total_nnz)
        self.tr = torch.zeros(3, dtype=torch.int64, device=dev)
        self.ed = _SingleEdge(eng, self.tr)
        rel = np.repeat(np.arange(dadj.num_relations), dadj.nnz)
        self.trip_all = torch.as_tensor(np.stack([np.concatenate(dadj.rows), rel, np.concatenate(dadj.cols)], 1),
                                        device=dev)
        self.eng, self.params, self.dadj = eng, params, dadj

        def body():
            self.ed.refresh()
            dv, _ = eng.value_grads(params, dadj, self.ed)
            s = torch.cat(dv)
            val, idx = torch.sort(s, descending=True, stable=True)   # == sorted(..., reverse=True)
            self.out_s = val[:self.k]
            self.out_t = self.trip_all[idx[:self.k]]

        self.tr.copy_(torch.zeros(3, dtype=torch.int64))
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):                 # warm-up: workspaces, allocator pools
            body()
        torch.cuda.current_stream(dev).wait_stream(side)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            body()

    def run(self, triples):
        n = len(triples)
        dev = self.eng.device
        tr_all = torch.as_tensor(np.asarray(triples, np.int64), device=dev)
        out_t = torch.empty(n, self.k, 3, dtype=torch.int64, device=dev)
        out_s = torch.empty(n, self.k, dtype=torch.float32, device=dev)
        for j in range(n):                            # launches only, no host synchronisation
            self.tr.copy_(tr_all[j])
            self.graph.replay()
            out_t[j].copy_(self.out_t)
            out_s[j].copy_(self.out_s)
        return out_t.cpu().numpy(), out_s.cpu().numpy()


# -- mask explainers -------------------------------------------------------------------------
class MaskAdam:
    """Keras 2.7 Adam on dense mask variables (TF ApplyAdam form, the iddgcn_adam_f32 kernel),
    moments and iteration count persisting across calls like the reference's shared optimizer."""

    def __init__(self, shape, device, learning_rate=1e-3, beta_1=0.9, beta_2=0.999, epsilon=1e-7):
        self.lr, self.b1, self.b2, self.eps = learning_rate, beta_1, beta_2, epsilon
        self.m = torch.zeros(shape, dtype=torch.float32, device=device)
        self.v = torch.zeros(shape, dtype=torch.float32, device=device)
        self.iterations = 0

    def apply(self, var, grad):
        self.iterations += 1
        f = np.float32
        t = f(self.iterations)
        alpha = f(self.lr) * np.sqrt(f(1) - f(self.b2) ** t) / (f(1) - f(self.b1) ** t)
        ops.adam(var, self.m, self.v, grad, alpha, self.b1, self.b2, self.eps, 0)


def structure_loss_grad(values, rel_of_entry, num_relations, target_ratios):
    """IDDGCN_explain.structure_loss (lines 30-41) and its gradient w.r.t. each masked value:
    ratios_r = sum(values of r) / sum(values); loss = mean((target - ratios)^2)."""
    counts = torch.zeros(num_relations, dtype=values.dtype, device=values.device).index_add_(0, rel_of_entry, values)
    total = counts.sum()
    ratios = counts / total
    target = torch.as_tensor(np.asarray(target_ratios), dtype=values.dtype, device=values.device)
    loss = ((target - ratios) ** 2).mean()
    dl_dratio = 2.0 * (ratios - target) / num_relations
    dl_dcount = (dl_dratio - (dl_dratio * ratios).sum()) / total        # d ratio_j / d count_r = (δ_jr - ratio_j)/C
    return loss, dl_dcount[rel_of_entry]


def _select(dadj, mvals, threshold, top_k):
    """Masked values above the threshold, relation by relation (skipping a relation whose kept
    (row, col) indices sum to 0, GnnExplainer.py:56-66), ranked descending, top_k."""
    mv = mvals.detach().cpu().numpy()
    trip, sc = [], []
    for r in range(dadj.num_relations):
        a, b = dadj.rel_offsets[r], dadj.rel_offsets[r + 1]
        keep = mv[a:b] > threshold
        rows, cols = dadj.rows[r][keep], dadj.cols[r][keep]
        if rows.sum() + cols.sum() == 0:
            continue
        trip.append(np.stack([rows, np.full(rows.shape, r, np.int64), cols], 1))
        sc.append(mv[a:b][keep])
    if not trip:
        return np.zeros((0, 3), np.int64), np.zeros((0,), np.float32)
    trip, sc = np.concatenate(trip), np.concatenate(sc)
    order = np.argsort(-sc, kind="stable")[:top_k]
    return trip[order], sc[order]


def mask_explainer(model, adjacency_data, test_triples, *, num_epochs=5, learning_rate=1e-3, threshold=0.2,
                   init_value=None, seed=123, target_ratios=None, top_k=10, optimizer=None, return_masks=False):
    """GNNExplainer.replica_step (GnnExplainer.py:26-74) and, with ``target_ratios``, the IDDGCN
    explainer's wgnnexplainer_step (IDDGCN_explain.py:43-118: loss = (pred_loss + struct_loss)/2).

    Returns (list of [k, 3] triples (head, rel, tail), list of [k] masked scores[, final masked
    values per triple]).  ``optimizer``: a MaskAdam to continue from (one is created otherwise)."""
    eng, params = _model_state(model)
    N, R = model.num_entities, model.num_relations
    dev = eng.device
    if init_value is None:
        init_value = np.random.default_rng(seed).standard_normal((N, N)).astype(np.float32)
    init = torch.as_tensor(np.asarray(init_value, np.float32).reshape(N, N), device=dev)
    masks = init.expand(R, N, N).contiguous()
    opt = optimizer or MaskAdam((R, N, N), dev, learning_rate)
    preds, scores, finals = [], [], []
    for tr in _as_triples(test_triples):
        comp = get_computation_graph(int(tr[0]), int(tr[1]), int(tr[2]), adjacency_data)
        adj_mats = get_adj_mats(comp, N, R)
        dadj = DeviceAdjacency(adj_mats, N, dev)
        rel_of = torch.as_tensor(np.repeat(np.arange(R), dadj.nnz), device=dev)
        flat = torch.as_tensor(np.concatenate([r * N * N + dadj.rows[r] * N + dadj.cols[r] for r in range(R)]),
                               device=dev)
        base = dadj.base_values
        ed = eng.edges(tr[None])
        dadj.set_values(base)
        before = eng.predict(params, dadj, ed)                        # unmasked prediction, constant
        for _ in range(num_epochs):
            sig = torch.sigmoid(masks.view(-1)[flat])
            mvals = base * sig
            dadj.set_values(mvals)
            dv, p = eng.value_grads(params, dadj, ed)                  # d pred / d masked values
            g = torch.cat(dv) * (-before / (p + 1e-5))                  # d(-before log(pred+1e-5))
            if target_ratios is not None:
                _, gs = structure_loss_grad(mvals, rel_of, R, target_ratios)
                g = (g + gs) * 0.5
            grad = torch.zeros(R * N * N, dtype=torch.float32, device=dev)
            grad[flat] = g * base * sig * (1.0 - sig)
            opt.apply(masks.view(-1), grad)
        mvals = base * torch.sigmoid(masks.view(-1)[flat])
        t_, s_ = _select(dadj, mvals, threshold, top_k)
        preds.append(t_)
        scores.append(s_)
        if return_masks:
            finals.append(mvals.cpu().numpy())
        masks.copy_(init.expand(R, N, N))                              # mask.assign(init_value)
    return (preds, scores, finals) if return_masks else (preds, scores)


def gnn_explainer(model, adjacency_data, test_triples, num_epochs=5, learning_rate=1e-3, threshold=0.2, **kw):
    """GnnExplainer.py defaults: 5 epochs, lr 1e-3, threshold 0.2, no structure loss."""
    return mask_explainer(model, adjacency_data, test_triples, num_epochs=num_epochs, learning_rate=learning_rate,
                          threshold=threshold, **kw)


def iddgcn_explainer(model, adjacency_data, test_triples, num_epochs=10, learning_rate=1e-3, threshold=0.15,
                     target_ratios=(0.4, 0.4, 0.1, 0.1), **kw):
    """IDDGCN_explain.py defaults: 10 epochs, lr 1e-3, threshold 0.15, ratios [.4, .4, .1, .1]."""
    if len(target_ratios) != model.num_relations:
        raise IddgcnError("target_ratios needs one entry per relation")
    return mask_explainer(model, adjacency_data, test_triples, num_epochs=num_epochs, learning_rate=learning_rate,
                          threshold=threshold, target_ratios=target_ratios, **kw)


def explanation_metrics(preds, gt, top=5, exp_num=10):
    """eval_test.py:15-39: Precision@top / Recall@top / F1@top of one explanation against its
    ground-truth triples (both orientations of each predicted triple count)."""
    preds_set = set(map(tuple, np.asarray(preds)))
    flip = np.flip(np.asarray(preds), axis=1)
    flip_set = set(map(tuple, flip))
    gt_set = set(map(tuple, np.asarray(gt)))
    pl, fl = list(preds_set), list(flip_set)
    tp = len(set(pl[:top]) & gt_set) + len(set(fl[:top]) & gt_set)
    fp = top - tp
    fn = exp_num - (len(preds_set & gt_set) + len(flip_set & gt_set))
    precision = tp / (tp + fp) if tp + fp > 0 else 0
    recall = tp / (tp + fn) if tp + fn > 0 else 0
    f1 = 2 * precision * recall / (precision + recall) if precision + recall > 0 else 0
    return precision, recall, f1
