"""Host-side graph build: per-relation adjacency and scored-edge layouts.

* ``get_adj_mats`` mirrors ``utils1.get_adj_mats`` (utils1.py:420-451): per
  relation, the sorted unique (obj, sbj) pairs with value 1.0, or the single
  placeholder (0,0)=0.0 for an empty relation, shaped (1, N, N) like the
  reference's reshaped ``tf.SparseTensor``.  The edge order is row-major
  sorted — exactly the order ``np.unique`` + ``tf.sparse.reorder`` produce —
  and it is the CSR order the SpMM kernel sums in.
* ``DeviceAdjacency`` holds, on the GPU, the batched CSR of every A_r (forward
  ``A_r·E``) and the batched CSR of every A_r^T (backward ``A_r^T·dAE_r``).
* ``ScoredEdges`` lays the scored triples (positives ++ negatives) out in HBM
  sorted by tail, so the tail-side gathers/scatters of every layer walk
  contiguous segments, and adds a head-sorted permutation for the head-side
  reductions.  All indices are validated here (int32, in range) so no kernel
  ever sees an out-of-range index.
* ``DeviceAdjacency.from_triples`` / ``ScoredEdges.from_triples`` build the same
  layouts on the GPU (include/iddgcn_graph.h: radix sorts, compaction, CSR
  pointers), bit-identical to the host build above; ``get_adj_mats(...,
  device=cuda)`` returns the device-built adjacency directly.
"""
import numpy as np
import torch

from ._lib import IddgcnError

INT32_MAX = 2 ** 31 - 1


class SparseAdj:
    """Host stand-in for the reference's (1, N, N) ``tf.SparseTensor``."""

    def __init__(self, indices, values, num_entities):
        self.indices = indices            # (nnz, 3) int64: [0, row, col]
        self.values = values              # (nnz,) float32
        self.dense_shape = (1, num_entities, num_entities)

    @property
    def rows(self):
        return self.indices[:, 1]

    @property
    def cols(self):
        return self.indices[:, 2]

    @property
    def nnz(self):
        return int(self.values.shape[0])


def _as_triples(data):
    if isinstance(data, torch.Tensor):
        data = data.cpu().numpy()
    data = np.asarray(data)
    if data.ndim == 3 and data.shape[0] == 1:
        data = data[0]
    if data.ndim != 2 or data.shape[1] != 3:
        raise IddgcnError(f"triples must be (B, 3), got {data.shape}")
    return data.astype(np.int64)


def get_adj_mats(data, num_entities, num_relations, device=None):
    """utils1.get_adj_mats (utils1.py:420-451) without TensorFlow.  With a GPU ``device`` the
    graph is built on the GPU and a DeviceAdjacency is returned (fit/predict take it in place of
    the list of SparseAdj)."""
    if device is not None and torch.device(device).type == "cuda":
        return DeviceAdjacency.from_triples(data, num_entities, num_relations, device)
    data = _as_triples(data)
    if data.size and (data[:, [0, 2]].min() < 0 or data[:, [0, 2]].max() >= num_entities):
        raise IddgcnError("entity index out of range [0, num_entities)")
    mats = []
    for r in range(num_relations):
        sel = data[data[:, 1] == r]
        if sel.shape[0] == 0:
            rc = np.zeros((1, 2), dtype=np.int64)
            val = np.zeros((1,), dtype=np.float32)
        else:
            # lexicographic (row, col) unique == np.unique(axis=0) == tf.sparse.reorder order
            key = sel[:, 0] * np.int64(num_entities) + sel[:, 2]
            key = np.unique(key)
            rc = np.stack([key // num_entities, key % num_entities], 1)
            val = np.ones((rc.shape[0],), dtype=np.float32)
        idx = np.concatenate([np.zeros((rc.shape[0], 1), dtype=np.int64), rc], 1)
        mats.append(SparseAdj(idx, val, num_entities))
    return mats


def _csr(rows, cols, n):
    order = np.lexsort((cols, rows))
    rows, cols = rows[order], cols[order]
    ptr = np.zeros(n + 1, dtype=np.int64)
    np.add.at(ptr, rows + 1, 1)
    return np.cumsum(ptr), cols, order


class DeviceAdjacency:
    """Batched CSR of every A_r (forward) and one merged CSR of all A_r^T (backward)."""

    def __init__(self, adj_mats, num_entities, device):
        N = num_entities
        self.num_entities = N
        self.num_relations = len(adj_mats)
        fptr, fcol, fval, fsrc = [], [], [], []
        bc, bm, bv = [], [], []
        off_f = 0
        any_val = False
        self.nnz = []
        self._rows, self._cols = [], []        # host copies, per relation, in the caller's entry order
        for r, a in enumerate(adj_mats):
            rows = np.asarray(a.rows, dtype=np.int64)
            cols = np.asarray(a.cols, dtype=np.int64)
            vals = np.asarray(a.values, dtype=np.float32)
            if rows.size and (rows.min() < 0 or rows.max() >= N or cols.min() < 0 or cols.max() >= N):
                raise IddgcnError("adjacency index out of range")
            any_val |= bool(np.any(vals != 1.0))
            p, c, o = _csr(rows, cols, N)
            fptr.append(p + off_f)
            fcol.append(c)
            fval.append(vals[o])
            fsrc.append(o + off_f)
            off_f += c.size
            bc.append(cols)
            bm.append(rows + r * N)
            bv.append(vals)
            self.nnz.append(int(rows.size))
            self._rows.append(rows)
            self._cols.append(cols)
        if off_f > INT32_MAX or N * len(adj_mats) > INT32_MAX:
            raise IddgcnError("adjacency too large for int32 offsets")
        # Backward: dE[c] += sum_r sum_{m: (m,c) in A_r} dAE[r][m].  One merged CSR of
        # [A_0^T | A_1^T | ...] over N rows whose column ids index the concatenated
        # dAE (R*N rows); inside a row entries run relation-major, then by m.
        bc, bm, bv = np.concatenate(bc), np.concatenate(bm), np.concatenate(bv)
        bptr, bcol, border = _csr(bc, bm, N)
        t = lambda x, dt: torch.as_tensor(np.ascontiguousarray(x).astype(dt), device=device)  # noqa: E731
        self.fwd_ptr, self.fwd_col = t(np.concatenate(fptr), np.int32), t(np.concatenate(fcol), np.int32)
        self.bwd_ptr, self.bwd_col = t(bptr, np.int32), t(bcol, np.int32)
        # values are all 1.0 unless a placeholder (0,0)=0 exists: pass them only then
        self.fwd_val = t(np.concatenate(fval), np.float32) if any_val else None
        self.bwd_val = t(bv[border], np.float32) if any_val else None
        self.total_nnz = off_f
        # entry k of the concatenated per-relation value lists (caller order) sits at CSR position
        # fwd_pos[k] of the forward CSR; the merged backward CSR reads value bwd_src[j]
        self.base_values = t(bv, np.float32)
        self.fwd_src = t(np.concatenate(fsrc), np.int64)
        self.fwd_pos = torch.empty_like(self.fwd_src)
        self.fwd_pos[self.fwd_src] = torch.arange(off_f, device=device)
        self.bwd_src = t(border, np.int64)
        self.rel_offsets = np.concatenate([[0], np.cumsum(self.nnz)]).astype(np.int64)
        self.device = device

    @classmethod
    def from_triples(cls, data, num_entities, num_relations, device):
        """get_adj_mats + __init__ on the GPU (iddgcn_build_adjacency): the entry order is the CSR
        order, so fwd_src / fwd_pos are the identity.  One host synchronisation (the counts)."""
        from . import ops
        tr = _device_triples(data, device)
        N, R = num_entities, num_relations
        out, nnz, nph, err = ops.build_adjacency(tr, N, R)
        if err:
            raise IddgcnError("entity index out of range [0, num_entities)")
        self = cls.__new__(cls)
        self.num_entities, self.num_relations, self.device = N, R, device
        self.fwd_ptr, self.bwd_ptr = out["fwd_ptr"], out["bwd_ptr"]
        self.fwd_col, self.bwd_col = out["fwd_col"][:nnz], out["bwd_col"][:nnz]
        self.fwd_val = out["fwd_val"][:nnz] if nph else None
        self.bwd_val = out["bwd_val"][:nnz] if nph else None
        self.total_nnz = nnz
        ends = self.fwd_ptr.view(R, N + 1)[:, [0, N]].cpu().numpy().astype(np.int64)
        self.nnz = [int(b - a) for a, b in ends]
        self.rel_offsets = np.concatenate([[0], np.cumsum(self.nnz)]).astype(np.int64)
        self.base_values = out["fwd_val"][:nnz]
        self.fwd_src = torch.arange(nnz, dtype=torch.int64, device=tr.device)
        self.fwd_pos = self.fwd_src
        self.bwd_src = out["bwd_src"][:nnz].long()
        self._rows = self._cols = None
        return self

    def _host_coo(self):
        ptr = self.fwd_ptr.view(self.num_relations, self.num_entities + 1).cpu().numpy().astype(np.int64)
        col = self.fwd_col.cpu().numpy().astype(np.int64)
        self._rows, self._cols = [], []
        for r in range(self.num_relations):
            deg = np.diff(ptr[r])
            self._rows.append(np.repeat(np.arange(self.num_entities, dtype=np.int64), deg))
            self._cols.append(col[ptr[r, 0]:ptr[r, -1]])

    @property
    def rows(self):
        """Per-relation row (obj) indices, host int64, entry order."""
        if self._rows is None:
            self._host_coo()
        return self._rows

    @property
    def cols(self):
        if self._cols is None:
            self._host_coo()
        return self._cols

    def set_values(self, values):
        """Replace the stored values (a (total_nnz,) GPU tensor in the caller's entry order, relation
        after relation) without rebuilding the CSR: ``adj * sigmoid(mask)`` of the explainers."""
        if values.shape != (self.total_nnz,):
            raise IddgcnError(f"values must have shape ({self.total_nnz},)")
        v = values.to(device=self.fwd_src.device, dtype=torch.float32)
        self.fwd_val = v[self.fwd_src].contiguous()
        self.bwd_val = v[self.bwd_src].contiguous()

    def bwd_columns(self, a, b):
        """The merged transposed CSR restricted to the entries whose column (flat relation-row r*N + i of
        dAE) lies in [a, b): (ptr, col, val) with every row's entries in their original order.  The
        row-partitioned transposed SpMM of data parallelism (Engine.spmm_shard) runs over it; cached per
        range (values refreshed by set_values are re-filtered)."""
        key = (int(a), int(b))
        cached = getattr(self, "_bwd_cols", None)
        if cached is not None and cached[0] == key and cached[1] is self.bwd_val:
            return cached[2]
        N = self.num_entities
        col = self.bwd_col.long()
        keep = (col >= a) & (col < b)
        rows = torch.repeat_interleave(torch.arange(N, device=col.device),
                                       (self.bwd_ptr[1:] - self.bwd_ptr[:-1]).long())
        counts = torch.bincount(rows[keep], minlength=N)
        ptr = torch.zeros(N + 1, dtype=torch.int32, device=col.device)
        ptr[1:] = torch.cumsum(counts, 0).to(torch.int32)
        out = (ptr, self.bwd_col[keep].contiguous(),
               None if self.bwd_val is None else self.bwd_val[keep].contiguous())
        self._bwd_cols = (key, self.bwd_val, out)
        return out

    def bwd_node_rows(self, a, b):
        """The merged transposed CSR restricted to the entries whose dAE row is node a <= i < b of ANY relation
        (column r*N + i): the transposed SpMM of a node-partitioned step (parallel.NodeShard) over the rows its
        rank owns, every output row's entries in their original order; cached per range."""
        key = (int(a), int(b))
        cached = getattr(self, "_bwd_nodes", None)
        if cached is not None and cached[0] == key and cached[1] is self.bwd_val:
            return cached[2]
        N = self.num_entities
        col = self.bwd_col.long()
        node = col % N
        keep = (node >= a) & (node < b)
        rows = torch.repeat_interleave(torch.arange(N, device=col.device),
                                       (self.bwd_ptr[1:] - self.bwd_ptr[:-1]).long())
        counts = torch.bincount(rows[keep], minlength=N)
        ptr = torch.zeros(N + 1, dtype=torch.int32, device=col.device)
        ptr[1:] = torch.cumsum(counts, 0).to(torch.int32)
        out = (ptr, self.bwd_col[keep].contiguous(),
               None if self.bwd_val is None else self.bwd_val[keep].contiguous())
        self._bwd_nodes = (key, self.bwd_val, out)
        return out

    def to_entry_order(self, csr_vals):
        """Per-entry quantity in forward-CSR order -> list of per-relation tensors in entry order."""
        flat = csr_vals[self.fwd_pos]
        return [flat[self.rel_offsets[r]:self.rel_offsets[r + 1]] for r in range(self.num_relations)]


def _device_triples(data, device):
    if isinstance(data, torch.Tensor) and data.is_cuda:
        t = data[0] if data.dim() == 3 and data.shape[0] == 1 else data
        if t.dim() != 2 or t.shape[1] != 3:
            raise IddgcnError(f"triples must be (B, 3), got {tuple(t.shape)}")
        return t.to(device=device, dtype=torch.int64).contiguous()
    return torch.as_tensor(np.ascontiguousarray(_as_triples(data)), device=device)


class ScoredEdges:
    """Scored triples (B, 3) laid out tail-sorted on the GPU.

    ``order[k]`` is the caller's row index of sorted position k; predictions
    are returned in the caller's order.
    """

    def __init__(self, triples, labels, num_entities, num_relations, device):
        tr = _as_triples(triples)
        T = tr.shape[0]
        if T > INT32_MAX:
            raise IddgcnError("too many scored edges for int32 indexing")
        h, r, t = tr[:, 0], tr[:, 1], tr[:, 2]
        if T and (min(h.min(), t.min()) < 0 or max(h.max(), t.max()) >= num_entities):
            raise IddgcnError("scored entity index out of range [0, num_entities)")
        if T and (r.min() < 0 or r.max() >= num_relations):
            raise IddgcnError("scored relation index out of range [0, num_relations)")
        order = np.argsort(t, kind="stable")
        self.order = order
        hs, rs, ts = h[order], r[order], t[order]
        tptr = np.searchsorted(ts, np.arange(num_entities + 1), side="left")
        hperm = np.argsort(hs, kind="stable")
        hptr = np.searchsorted(hs[hperm], np.arange(num_entities + 1), side="left")
        g = lambda x, dt: torch.as_tensor(np.ascontiguousarray(x).astype(dt), device=device)  # noqa: E731
        self.T = T
        self.h, self.r, self.t = g(hs, np.int32), g(rs, np.int32), g(ts, np.int32)
        self.tptr, self.hperm, self.hptr = g(tptr, np.int32), g(hperm, np.int32), g(hptr, np.int32)
        self.y = None if labels is None else g(np.asarray(labels, dtype=np.float32)[order], np.float32)
        self.inv = g(np.argsort(order, kind="stable"), np.int64)

    @classmethod
    def from_triples(cls, triples, labels, num_entities, num_relations, device):
        """__init__ on the GPU (iddgcn_build_scored_edges): same arrays, bit-identical; ``order``
        is a GPU int32 tensor here.  One host synchronisation (the error flag)."""
        from . import ops
        tr = _device_triples(triples, device)
        if tr.shape[0] > INT32_MAX:
            raise IddgcnError("too many scored edges for int32 indexing")
        lab = None
        if labels is not None:
            lab = torch.as_tensor(np.asarray(labels, dtype=np.float32) if not isinstance(labels, torch.Tensor)
                                  else labels, device=device).to(torch.float32).reshape(-1).contiguous()
        o, err = ops.build_scored_edges(tr, lab, num_entities, num_relations)
        if err & 1:
            raise IddgcnError("scored entity index out of range [0, num_entities)")
        if err & 2:
            raise IddgcnError("scored relation index out of range [0, num_relations)")
        self = cls.__new__(cls)
        self.T = tr.shape[0]
        self.h, self.r, self.t = o["h"], o["r"], o["t"]
        self.tptr, self.hperm, self.hptr = o["tptr"], o["hperm"], o["hptr"]
        self.y, self.inv = o["y"], o["inv"]
        self.order = None
        return self

    def unsort(self, x):
        """Sorted-order per-edge tensor -> caller's order."""
        return x[self.inv]
