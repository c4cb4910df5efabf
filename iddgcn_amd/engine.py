"""Step engine: the whole IDDGCN training / inference step as HIP launches.

Formulation.  The reference evaluates every layer per
scored edge (IDDGCN.py:60-79).  Three exact identities move most of it to the
node level (N rows instead of T = B_pos + B_neg rows):

  1. ``AE_r = A_r·E`` does not depend on the layer input (the layer is always
     fed ``all_e``, IDDGCN.py:243/256/269) -> one SpMM per relation per step;
  2. ``AE_r[idx]·K_r == (AE_r·K_r)[idx]`` -> ``P_r^l = AE_r·K_r^l`` per node;
  3. the head chain ``x_h^l`` (and the dynamic weights ``w^l``, computed from
     the head only, IDDGCN.py:66) depend on the head entity alone -> computed
     once per node as ``X^l``.

What stays per edge is the tail chain: layer 1 is a pure gather-combine of
node tables, layers 2-3 need ``x_t^{l-1}·S^l`` (MFMA) fused with the gather of
``P_r^l[t]`` scaled by ``w^l[h]`` and the sigmoid.  The backward mirrors this:
edge-level MFMA GEMMs for ``dx·S^T`` and ``dS``, deterministic segmented
reductions for every scatter, node-level MFMA GEMMs for the rest.

Parameters live in ONE flat fp32 buffer (and so do their gradients), so Adam
is two launches and data-parallel training needs one all-reduce per step.
"""
import contextlib

import numpy as np
import torch

from . import _lib as L
from . import ops
from .graph import DeviceAdjacency, ScoredEdges

NUM_LAYERS = 3


def param_layout(N, R, D):
    """(name, shape, sparse_form) in flat-buffer order.  E and rel use the
    Keras sparse-Adam form (their TF gradients are IndexedSlices)."""
    lay = [("E", (N, D), True), ("rel", (R, D), True)]
    for l in range(1, NUM_LAYERS + 1):
        lay += [(f"K{l}", (R, D, D), False), (f"S{l}", (D, D), False),
                (f"Wa{l}", (D, R), False), (f"ba{l}", (R,), False)]
    return lay


class FlatParams:
    """A flat fp32 buffer with named views (parameters or their gradients).

    ``buf`` is ``[flat | loss]``: one float past the parameters holds the step's loss sum when the
    buffer carries gradients, so a data-parallel step all-reduces gradients and loss IN PLACE in
    one buffer (parallel.BucketedAllReduce), no bucket copies.  E comes first, so ``buf[N*D:]`` (all
    small gradients + the loss) and row ranges of ``E`` are contiguous buckets."""

    def __init__(self, N, R, D, device):
        self.N, self.R, self.D = N, R, D
        self.layout = param_layout(N, R, D)
        total = sum(int(np.prod(s)) for _, s, _ in self.layout)
        self.buf = torch.zeros(total + 1, dtype=torch.float32, device=device)
        self.flat = self.buf[:total]
        self.loss = self.buf[total:]
        self.views, off = {}, 0
        self.n_sparse = 0
        for name, shape, sparse in self.layout:
            n = int(np.prod(shape))
            self.views[name] = self.flat[off:off + n].view(shape)
            if sparse:
                self.n_sparse = off + n
            off += n

    def __getitem__(self, k):
        return self.views[k]

    def load(self, d):
        for name, shape, _ in self.layout:
            if name in d:
                src = torch.as_tensor(np.asarray(d[name], dtype=np.float32).reshape(shape))
                self.views[name].copy_(src)

    def to_numpy(self):
        return {k: v.detach().cpu().numpy().copy() for k, v in self.views.items()}


class KerasAdam:
    """Keras 2.7 Adam (lr=1e-3, b1=.9, b2=.999, eps=1e-7) over a FlatParams."""

    def __init__(self, params, learning_rate=1e-3, beta_1=0.9, beta_2=0.999, epsilon=1e-7):
        self.lr, self.b1, self.b2, self.eps = learning_rate, beta_1, beta_2, epsilon
        self.m = torch.zeros_like(params.flat)
        self.v = torch.zeros_like(params.flat)
        self._n_e = params["E"].numel()
        self.iterations = 0

    def alpha_at(self, t):
        """lr_t of iteration t, computed in fp32 as TF does."""
        f = np.float32
        t = f(t)
        b1p, b2p = f(self.b1) ** t, f(self.b2) ** t
        return f(self.lr) * np.sqrt(f(1) - b2p) / (f(1) - b1p)

    def apply(self, params, grads):
        self.iterations += 1
        alpha = self.alpha_at(self.iterations)
        self._apply_range(params, grads, 0, params.flat.numel(), alpha)

    def _apply_range(self, params, grads, lo, hi, alpha):
        """The update of flat elements [lo, hi) (sparse form below params.n_sparse, dense above); the update is
        elementwise, so any partition of the buffer gives bitwise the whole-buffer result."""
        ns = params.n_sparse
        for a, b, sparse in ((lo, min(hi, ns), 1), (max(lo, ns), hi, 0)):
            if a < b:
                ops.adam(params.flat[a:b], self.m[a:b], self.v[a:b], grads.flat[a:b], alpha, self.b1, self.b2,
                         self.eps, sparse)

    def apply_overlapped(self, params, grads, comm):
        """apply() after a data-parallel backward, bucket by bucket: each all-reduced bucket of ``grads.buf``
        (parallel.BucketedAllReduce.finish_each, in hand-over order) gets its parameters' update as soon as its
        sum has landed, so the update of the small weights and of dE's first row chunks runs while the later
        chunks are still on the wire; the elements no bucket covered are updated after the last."""
        self.iterations += 1
        alpha = self.alpha_at(self.iterations)
        n, base = params.flat.numel(), grads.buf.data_ptr()
        done = []

        def on_bucket(view):
            off = (view.data_ptr() - base) // view.element_size()
            if view.dtype != grads.buf.dtype or not 0 <= off < n:
                return
            hi = min(off + view.numel(), n)
            self._apply_range(params, grads, off, hi, alpha)
            done.append((off, hi))

        comm.finish_each(on_bucket)
        pos = 0
        for a, b in sorted(done) + [(n, n)]:
            if a > pos:
                self._apply_range(params, grads, pos, a, alpha)
            pos = max(pos, b)


    def apply_owned(self, params, grads, comm, rs_e, e_lo, e_hi):
        """apply() after a node-partitioned backward whose dE was reduce-scattered to the row owners
        (Engine._backward_rows with e_owner; round 5): the small gradients' buckets (everything past E, all-reduced)
        are updated as their sums land, then this rank's E rows — flat elements [e_lo, e_hi) — once ``rs_e`` (the
        reduce-scatter handle) completes.  The other E rows and their moments are left to their owners (the
        caller all-gathers E); the update being elementwise, the owners' rows together are the whole update."""
        self.iterations += 1
        alpha = self.alpha_at(self.iterations)
        n, base = params.flat.numel(), grads.buf.data_ptr()
        n_e = params["E"].numel()

        def on_bucket(view):
            off = (view.data_ptr() - base) // view.element_size()
            if view.dtype == grads.buf.dtype and n_e <= off < n:
                self._apply_range(params, grads, off, min(off + view.numel(), n), alpha)

        comm.finish_each(on_bucket)
        rs_e.wait()
        if e_hi > e_lo:
            self._apply_range(params, grads, e_lo, e_hi, alpha)

    def gather_owned_state(self, shard):
        """After apply_owned steps the Adam moments of E are partitioned by rows: each rank's m / v hold its own rows
        [shard.a, shard.b) only (the others stay at their last all-reduced state).  All-gather them so every rank holds
        the whole optimizer state (a checkpoint, or a switch back to a replicated update); the rows are the owners'
        bitwise."""
        for t in (self.m, self.v):
            shard.all_gather(t[:self._n_e].view(shard.N, -1))

    def apply_table(self, params, grads, alpha_table, step):
        """apply() with alpha = alpha_table[step] read on the device (HIP-graph replay); the caller
        advances ``step`` and, after the replays, ``iterations``."""
        ns = params.n_sparse
        ops.adam_table(params.flat[:ns], self.m[:ns], self.v[:ns], grads.flat[:ns], alpha_table, step, self.b1,
                       self.b2, self.eps, 1)
        ops.adam_table(params.flat[ns:], self.m[ns:], self.v[ns:], grads.flat[ns:], alpha_table, step, self.b1,
                       self.b2, self.eps, 0)


class GraphedTrainStep:
    """Engine.train_step + Keras Adam + loss record captured once in a HIP graph and replayed per
    epoch: one graph launch per step instead of ~61 host-issued launches (fit() on the reference's
    fold-sized graphs, N=845 / T=40k, is launch-bound).  Bitwise the same step: the Adam alpha of
    each iteration comes from the host's float32 formula, tabulated for the ``n_steps`` iterations
    after ``opt.iterations`` and indexed by a device counter.  Single process only (no all-reduce
    inside the graph).  Needs a prior eager step on the same (engine, edges) so every workspace
    exists before capture."""

    def __init__(self, eng, params, grads, opt, adj, ed, n_steps, t_global=None):
        dev = eng.device
        t0 = opt.iterations
        self.opt, self.n = opt, n_steps
        self.alpha = torch.as_tensor(np.array([opt.alpha_at(t0 + k + 1) for k in range(n_steps)], np.float32),
                                     device=dev)
        self.step = torch.zeros(1, dtype=torch.int32, device=dev)
        self.losses = torch.zeros(max(n_steps, 1), dtype=torch.float32, device=dev)
        self.done = 0
        ws = eng.workspace(ed.T, True)
        self.ws = ws        # the captured pointers live as long as the graph (Engine may evict its copy)

        def body():
            eng._t_global = t_global
            eng.forward(params, adj, ed, ws, True)
            eng.backward(params, grads, adj, ed, ws)
            opt.apply_table(params, grads, self.alpha, self.step)
            ops.step_advance(self.step, self.losses, grads.loss)

        torch.cuda.synchronize(dev)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            body()

    def replay(self):
        """One training step; returns the device scalar holding its loss sum."""
        if self.done >= self.n:
            raise L.IddgcnError("GraphedTrainStep: alpha table exhausted")
        self.graph.replay()
        self.done += 1
        self.opt.iterations += 1
        return self.losses[self.done - 1]


class Workspace:
    """Every device buffer one step needs, sized for (N, R, D, T).

    Edge tables: only the three tail activations x^1..x^3 (T x D each).  The backward writes the
    edge-level gradients over them in place: DistMult writes do^3 over x^3, and the layer-l backward
    GEMM writes do^{l-1} = (do^l S^T) * x^{l-1}(1 - x^{l-1}) over its own sigma' operand x^{l-1}
    (each element is read before it is written, by the same lanes).  3 T x D tables instead of 5:
    123 GB instead of 205 GB at config 4 (T = 40M, D = 256)."""

    def __init__(self, N, R, D, T, device, train=True, edge_dtype=torch.float32):
        f = dict(dtype=torch.float32, device=device)
        e = lambda *s: torch.empty(*s, **f)  # noqa: E731
        self.AE = e(R, N, D)
        self.ES1 = e(N, D)                      # E·S^1 (layer-1 x·S at node level)
        self.P = e(NUM_LAYERS, R, N, D)         # P_r^l = AE_r·K_r^l
        self.X = e(NUM_LAYERS, N, D)            # head chain X^1..X^3
        self.Ssm = e(NUM_LAYERS, N, R)
        self.W = e(NUM_LAYERS, N, R)
        # tail chain x^1..x^3 (then, training, do^3..do^1); bf16 in the bf16-feature mode
        self.xt = torch.empty(NUM_LAYERS, T, D, dtype=edge_dtype, device=device)
        self.Wedge = e(NUM_LAYERS, T, R)        # W^l[h_e]: per-edge copy of the dynamic weights
        self.p = e(T)
        self.s = e(T)                           # pre-sigmoid DistMult logits (IDDGCN.py:108)
        self.nb_dm = ops.distmult_blocks(T)
        self.train = train
        if not train:
            return
        self.dWedge = e(T, R)
        self.dOn_a = e(N, D)                    # node-level grads, ping-pong
        self.dOn_b = e(N, D)
        self.dP = e(R, N, D)
        self.dAE = e(R, N, D)
        self.dES = e(N, D)
        self.dz = e(N, R)
        self.dwh = e(N, R)                      # <head seed, P_r> per node (fused R = 8 tail + head backward)
        self.WaT = e(R, D)
        self.drel_slab = e(self.nb_dm * R * D)
        self.loss_slab = e(self.nb_dm)
        # partials of the edge TN, or of one batched launch of up to L.TN_BATCH node-level TNs
        tn = max(ops.tn_blocks(T, D), min(256, L.TN_BATCH * ops.tn_blocks(N, D)), ops.tn_blocks(N, D),
                 ops.sigma_tn_slab_floats(T, D) // (D * D) if D == 256 else 1)
        self.tn_slab = e(tn * D * D)
        self.narrow_slab = e((ops.tn_narrow_blocks(N) + 1) * (D + 1) * R)


GEMM_MODES = {"exact": L.GEMM_EXACT_F32, "split": L.GEMM_SPLIT_F16, "bf16x3": L.GEMM_BF16X3}
PROJ_MODES = {"exact": L.GEMM_EXACT_F32, "split": L.GEMM_SPLIT_F16, "exact4": L.GEMM_F32_4CHAIN,
              "bf16x3": L.GEMM_BF16X3}


class Engine:
    """Runs forward / backward / Adam for one (graph, scored-edge batch).

    ``gemm`` selects the operand precision of the D=256 MFMA GEMMs, passed with every GEMM call
    (include/iddgcn.h IDDGCN_GEMM_*, ABI 6: no process-global state, so engines in different modes may
    run side by side on different streams or threads): "exact" (default) runs v_mfma_f32_32x32x2_f32,
    bitwise an fmaf chain — the reference's fp32 arithmetic; "bf16x3" splits every fp32 operand EXACTLY
    into three bf16 pieces (24 significant bits: the whole fp32 value) and sums the six piece products of
    order >= 2^-16 on bf16 MFMAs with fp32 accumulation (dropped terms <= 2^-23 |a w| per product, fp32's own
    product rounding is 2^-24): fp32 arithmetic at 2.7x the f32 MFMA rate; "split" splits every fp32 operand
    into two fp16 halves with power-of-two row/column scales (22 significant bits, 3 f16 MFMAs per k-step), an
    opt-in faster mode.  Other widths and all non-GEMM kernels are exact f32 in every mode.
    """

    def __init__(self, num_entities, num_relations, dim, device=None, gemm="exact", features="f32", planes=True,
                 edge_mfma="hilo"):
        if dim not in (32, 64, 128, 256):
            raise L.IddgcnError("embedding dim must be one of 32, 64, 128, 256")
        if features not in ("f32", "bf16"):
            raise L.IddgcnError("features must be 'f32' or 'bf16'")
        if features == "bf16" and dim != 256:
            raise L.IddgcnError("the bf16-feature mode is D=256 only")
        # bf16-feature mode (BASELINE config 5, perf only): the edge tables x^l / do^l stored as bf16 and
        # the edge GEMMs on bf16 MFMA; node tables, weights, accumulation and epilogues stay fp32
        self.features = features
        self.edge_dtype = torch.bfloat16 if features == "bf16" else torch.float32
        # operands of the bf16 edge GEMMs (include/iddgcn.h IDDGCN_GEMM_BF16): "hilo" keeps the weights (and the R = 8
        # combine's node rows / coefficients) as a bf16 hi + lo pair, 16 significant bits, so the edge tables' bf16
        # storage is the only rounding beyond fp32; "bf16" rounds every MFMA operand to bf16 once (one product per
        # term, fp32 accumulation: config 5's "bf16 features with MFMA XW" as autocast runs it)
        if edge_mfma not in ("hilo", "bf16"):
            raise L.IddgcnError("edge_mfma must be 'hilo' or 'bf16'")
        if edge_mfma == "bf16" and features != "bf16":
            raise L.IddgcnError("edge_mfma='bf16' needs features='bf16' (bf16 edge tables)")
        self.edge_mfma = edge_mfma
        self.fuse_sigma_tn = True
        # bf16 edge tables at R = 8, D = 256: the tail reduction adds the head chain's node terms (tail_seg_reduce_head)
        # and head_dz finishes the head side; False runs the plain tail reduction + head_bwd_node (A/B, tests)
        self.fuse_tail_head = True
        if not 1 <= num_relations <= 8:
            raise L.IddgcnError("num_relations must be in [1, 8]")
        if gemm not in GEMM_MODES:
            raise L.IddgcnError(f"gemm must be one of {sorted(GEMM_MODES)}")
        self.N, self.R, self.D = num_entities, num_relations, dim
        self.gemm = gemm
        # pre-split tail tables x^1, x^2 (include/iddgcn.h IDDGCN_PLANES_*): their producers (layer-1
        # combine, layer-2 forward GEMM) write [hi | lo] fp16 rows once, so the forward GEMMs of layers 2-3,
        # the dS TN GEMMs and the sigma' backward skip their per-tile conversion (see use_planes)
        self.planes = planes
        self.device = torch.device("cuda") if device is None else torch.device(device)
        if self.device.type != "cuda":
            raise L.IddgcnError("IDDGCN engine runs on the GPU only (no CPU fallback)")
        L.lib()  # fail loudly now if the HIP library is missing
        self._ws = {}
        self.probe = None      # {name: [(start_event, end_event), ...]} when timing kernels

    @property
    def gemm(self):
        return self._gemm

    @gemm.setter
    def gemm(self, mode):
        if mode not in GEMM_MODES:
            raise L.IddgcnError(f"gemm must be one of {sorted(GEMM_MODES)}")
        self._gemm = mode

    _proj_gemm = None

    @property
    def proj_gemm(self):
        """Precision of the node-level projections (plain row GEMMs over N rows: P_r^l = AE_r K_r^l, E S^1 and
        the backward's dAE_r = dP_r K_r^T).  Default: "exact4" (f32 MFMA, four interleaved accumulation
        chains) in the exact mode — AE_r sums ~20 entity rows, P reaches |1e3| at the reference's init, and a
        256-long fp32 chain there was the largest error of the logits (tools/logit_error_probe.py) — else
        the engine's ``gemm``."""
        if self._proj_gemm is not None:
            return self._proj_gemm
        if self._gemm == "bf16x3" and self.D < 256:
            return "exact4"
        return "exact4" if self._gemm == "exact" else self._gemm

    _row_gemm = None

    @property
    def row_gemm(self):
        """Precision of the other row GEMMs (the tail / head chains and their backward): the engine's ``gemm``,
        except at D < 256 in the exact mode, where the register-staged kernel takes "exact4" for every form (the
        four-chain accumulation costs nothing there and keeps the trained-weight logits of the reference's
        64-wide model further inside the 1e-4 bar).  Settable (None = this default), as ``proj_gemm`` is: a second
        summation order for the training-drift measurement (tools/fold_order_sensitivity.py)."""
        if self._row_gemm is not None:
            return self._row_gemm
        return "exact4" if (self._gemm in ("exact", "bf16x3") and self.D < 256) else self._gemm

    @row_gemm.setter
    def row_gemm(self, mode):
        if mode is not None and mode not in PROJ_MODES:
            raise L.IddgcnError(f"row_gemm must be None or one of {sorted(PROJ_MODES)}")
        self._row_gemm = mode

    @proj_gemm.setter
    def proj_gemm(self, mode):
        if mode is not None and mode not in PROJ_MODES:
            raise L.IddgcnError(f"proj_gemm must be None or one of {sorted(PROJ_MODES)}")
        self._proj_gemm = mode

    @property
    def edge_gemm(self):
        """Precision of the edge-level row GEMMs (the tail chain's forward and sigma' backward): "bf16" with
        edge_mfma="bf16" (bf16 edge tables), else ``row_gemm``."""
        return "bf16" if self.edge_mfma == "bf16" else self.row_gemm

    @property
    def sigma_tn_fused(self):
        """A layer's dS TN and sigma' backward GEMM run as one pass over do^l and x^{l-1} (ops.sigma_tn) instead of two:
        bf16 edge tables at D = 256 (config 5's mode, ABI 11; the sigma' weights as ``edge_gemm`` takes them), and fp32
        tables in the bf16x3 mode at D = 256 (the headline, ABI 12).  ``fuse_sigma_tn`` = False keeps the two kernels,
        for A/B."""
        if not (self.fuse_sigma_tn and self.D == 256):
            return False
        return self.features == "bf16" or (self.edge_gemm == "bf16x3" and self._gemm == "bf16x3")

    @property
    def use_planes(self):
        """x^1, x^2 are stored pre-split: split GEMM mode at D = 256 with fp32 features, R <= 2 (the
        gathered forward's planes form)."""
        return self.planes and self.gemm == "split" and self.D == 256 and self.features == "f32" and self.R <= 2

    @contextlib.contextmanager
    def _mark(self, name):
        """Bracket one launch with HIP events on the current stream (bench.py roofline)."""
        if self.probe is None:
            yield
            return
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        yield
        b.record()
        self.probe.setdefault(name, []).append((a, b))

    # -- setup --------------------------------------------------------------
    def adjacency(self, adj_mats):
        if isinstance(adj_mats, DeviceAdjacency):
            return adj_mats
        return DeviceAdjacency(adj_mats, self.N, self.device)

    def edges(self, triples, labels=None):
        """Scored-edge layout, built on the GPU (iddgcn_build_scored_edges)."""
        return ScoredEdges.from_triples(triples, labels, self.N, self.R, self.device)

    def release(self):
        """Drop the cached workspaces (their device memory goes back to torch's caching allocator): a
        predict workspace and a training workspace of a 40M-edge batch do not fit one GPU together."""
        self._ws = {}

    def workspace(self, T, train):
        key = (T, train)
        if key not in self._ws:
            self._ws = {k: v for k, v in self._ws.items() if k[1] != train}  # keep one per mode
            self._ws[key] = Workspace(self.N, self.R, self.D, T, self.device, train, self.edge_dtype)
        return self._ws[key]

    # -- forward ------------------------------------------------------------
    # backward: the layer-2/3 tail reductions (HBM-bound) on a side stream beside the exact-mode dS TN (MFMA-bound,
    # 151 VGPRs: room for two more waves per SIMD)
    overlap = False
    _side = None

    def _side_stream(self):
        if self._side is None or self._side.device != torch.cuda.current_stream().device:
            self._side = torch.cuda.Stream(device=self.device)
        return self._side

    node_shard = None      # parallel.RelationShard: per-relation node tables split over the ranks
    row_shard = None       # parallel.NodeShard: node rows split over the ranks, scored edges by tail (round 4)
    # parallel.RelationShard used for the two SpMMs only (node GEMMs replicated): A_r·E row-partitioned and
    # all-gathered, dAE reduce-scattered to the row owners before a transposed SpMM over their columns
    spmm_shard = None

    def forward(self, P, adj, ed, ws, train):
        if self.row_shard is not None:
            return self._forward_rows(P, adj, ed, ws, train)
        N, R, D, T = self.N, self.R, self.D, ed.T
        E = P["E"]
        # every GEMM call carries this engine's operand precision: pn for the plain node-level projections, pr for
        # the other row GEMMs
        pn = dict(precision=self.proj_gemm)
        pr = dict(precision=self.row_gemm)      # (the other row GEMMs)
        sh = self.node_shard
        if sh is None and self.spmm_shard is not None:
            # row-partitioned A_r·E (every rank holds E): this rank's (relation, row) pieces, then all-gather
            ss = self.spmm_shard
            for r, n0, n1 in ss.pieces():
                ops.spmm_csr(adj.fwd_ptr[r * (N + 1) + n0:r * (N + 1) + n1 + 1], adj.fwd_col, adj.fwd_val, E,
                             ws.AE[r][n0:n1].view(1, n1 - n0, D), 1, n1 - n0)
            ss.all_gather(ws.AE.view(R * N, D))
            proj = [(ws.AE[r], P[f"K{l + 1}"][r], ws.P[l, r], pn) for l in range(NUM_LAYERS) for r in range(R)]
        elif sh is None:
            # AE_r = A_r·E, all relations in one launch (IDDGCN.py:69-70)
            ops.spmm_csr(adj.fwd_ptr, adj.fwd_col, adj.fwd_val, E, ws.AE, R, N)
            # P_r^l = AE_r·K_r^l (node-level form of IDDGCN.py:71-72,76-77) and, layer 1, x·S1 at node
            # level for both sides (inputs E[h], E[t]): independent GEMMs, batched (one launch below D=256)
            proj = [(ws.AE[r], P[f"K{l + 1}"][r], ws.P[l, r], pn) for l in range(NUM_LAYERS) for r in range(R)]
        else:
            # relation-sharded: this rank's (relation, node-row) pieces of AE_r and P_r^l, then all-gather P
            proj = []
            for r, n0, n1 in sh.pieces():
                ops.spmm_csr(adj.fwd_ptr[r * (N + 1) + n0:r * (N + 1) + n1 + 1], adj.fwd_col, adj.fwd_val, E,
                             ws.AE[r][n0:n1].view(1, n1 - n0, D), 1, n1 - n0)
                proj += [(ws.AE[r][n0:n1], P[f"K{l + 1}"][r], ws.P[l, r][n0:n1], pn) for l in range(NUM_LAYERS)]
        proj.append((E, P["S1"], ws.ES1, pn))
        nb = L.ROWGEMM_BATCH
        for i in range(0, len(proj), nb):
            ops.rowgemm_batched(proj[i:i + nb])
        if sh is not None:
            for l in range(NUM_LAYERS):
                sh.all_gather(ws.P[l].view(R * N, D))
        ops.alpha_fwd(E, P["Wa1"], P["ba1"], ws.Ssm[0], ws.W[0])
        ops.gather_rows(ws.W[0], ed.h, ws.Wedge[0])
        ops.combine(ws.ES1, ws.W[0], ws.P[0], ws.X[0])
        pl = self.use_planes
        ops.combine(ws.ES1, ws.Wedge[0], ws.P[0], ws.xt[0], y_idx=ed.t, v_idx=ed.t, planes_out=pl)
        # layers 2, 3
        for l in (1, 2):
            S = P[f"S{l + 1}"]
            ops.alpha_fwd(ws.X[l - 1], P[f"Wa{l + 1}"], P[f"ba{l + 1}"], ws.Ssm[l], ws.W[l])
            ops.gather_rows(ws.W[l], ed.h, ws.Wedge[l])
            if R > 2 and D == 256:
                # head chain at node level, many relations: X^{l-1}·S into ES1 (free once the layer-1 combines above
                # have read it), then the row-aligned combine sigma(Y + sum_r W_r P_r) — every node row's own 8 V rows,
                # which the fused GEMM's gathered-V epilogue (built for tail runs) stages through its capped slabs
                # one row at a time: config 5 4.5 ms -> 0.6 + 1.9 ms
                ops.rowgemm(ws.X[l - 1], S, ws.ES1, **pr)
                ops.combine(ws.ES1, ws.W[l], ws.P[l], ws.X[l])
            else:
                ops.rowgemm(ws.X[l - 1], S, ws.X[l], coef=ws.W[l], V=ws.P[l], v_rel_stride=N * D,
                            act=L.ACT_SIGMOID, **pr)
            with self._mark("tail_fwd_gemm"):
                ops.rowgemm(ws.xt[l - 1], S, ws.xt[l], coef=ws.Wedge[l], V=ws.P[l], v_idx=ed.t,
                            v_rel_stride=N * D, act=L.ACT_SIGMOID,
                            planes=(L.PLANES_A | (L.PLANES_C if l == 1 else 0)) if pl else 0, precision=self.edge_gemm)
        # DistMult (+ BCE and backward seed when training)
        if train:
            # one pass over head segments: p / loss / drel partials, the tail seed do^3 (per edge)
            # and the head seed dO^3[n] = X3(1-X3) * sum_{h_e=n} ds_e rel[r_e] * x3_e
            if self._pred_seed is None:        # Keras BCE, x 1/num_entities (IDDGCN.py:161-168)
                scale, y = 1.0 / (float(self._t_global or T) * float(N)), ed.y
            else:                              # d(scale * sum_e p_e): the explainers' seed
                scale, y = float(self._pred_seed), None
            # do^3 is written over x^3 in place (each edge row is read, then written, by the same lanes)
            ops.distmult_bce_heads(ed.hptr, ed.hperm, ws.X[2], ws.xt[2], ed.r, P["rel"], y, ws.xt[2], ws.dOn_a,
                                   ws.drel_slab, ws.loss_slab, scale=scale, p_out=ws.p if self._want_p else None,
                                   s_out=ws.s if self._want_p else None)
        else:
            ops.distmult_bce(ws.X[2], ed.h, ws.xt[2], ed.r, P["rel"], p_out=ws.p, s_out=ws.s)

    _t_global = None
    _want_p = False        # per-edge probabilities are only materialised for loss_and_grads
    _pred_seed = None      # None: BCE seed; a float: gradient of pred_seed * sum_e p_e

    # -- backward -----------------------------------------------------------
    def backward(self, P, G, adj, ed, ws, comm=None, e_owner=False):
        """Gradients of the step into G (and the loss sum into G.loss).  ``comm`` (data parallel,
        parallel.BucketedAllReduce) gets each contiguous piece of G.buf as soon as it is final: all
        small gradients + the loss after the layer loop, then row chunks of dE as the transposed SpMM
        produces them, so the all-reduce of the large dE overlaps the SpMM of the next chunk.  ``e_owner``
        (node-partitioned steps only): dE is reduce-scattered to the row owners instead (returns the handle)."""
        if self.row_shard is not None:
            return self._backward_rows(P, G, adj, ed, ws, comm, e_owner)
        N, R, D = self.N, self.R, self.D
        pk, pn, pr = dict(precision=self.gemm), dict(precision=self.proj_gemm), dict(precision=self.row_gemm)
        dOn, dOn_next = ws.dOn_a, ws.dOn_b      # head seed dO^3, written by distmult_bce_heads
        if self.node_shard is not None:
            ws.dAE.zero_()                      # rows other ranks own stay 0 in the dE SpMM below
        pl = self.use_planes                    # x^1, x^2 are planes tables (forward)
        for l in (2, 1, 0):                     # layer index l -> reference layer l+1
            Wl, Pl, Sl = ws.W[l], ws.P[l], P[f"S{l + 1}"]
            do = ws.xt[l]                       # do^{l+1}, written over x^{l+1}
            # tail side: dP (tail part), dWedge, and for layer 1 the dES tail part.  With `overlap` (layers
            # 2-3) the HBM-bound reduction runs on a side stream beside the MFMA-bound dS TN and sigma'
            # GEMM (it reads do, P, Wedge and writes dP, dWedge: nothing those two touch); the side stream
            # first waits for everything queued so far (the previous layer's readers of dP), and the
            # main stream waits for it before the head-side work that reads dP, dWedge
            side = self._side_stream() if (self.overlap and l > 0) else None
            # bf16 edge tables at R = 8, D = 256 (config 5): the tail reduction on MFMAs adds the head chain's node terms
            # (Wl[n] dO[n] into dP, dO[n] into dES) before its store, so the head backward below skips them
            fused = self.fuse_tail_head and self.features == "bf16" and R == 8 and D == 256 and self.node_shard is None
            if side is not None:
                side.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(side):
                    if fused:
                        ops.tail_seg_reduce_head(ed.tptr, ws.Wedge[l], do, Pl, ws.dP, ws.dWedge, dOn, Wl, ws.dwh)
                    else:
                        ops.tail_seg_reduce(ed.tptr, None, ws.Wedge[l], do, Pl, ws.dP, ws.dWedge)
            elif fused:
                ops.tail_seg_reduce_head(ed.tptr, ws.Wedge[l], do, Pl, ws.dP, ws.dWedge, dOn, Wl, ws.dwh,
                                         dsum=ws.dES if l == 0 else None)
            else:
                ops.tail_seg_reduce(ed.tptr, None, ws.Wedge[l], do, Pl, ws.dP, ws.dWedge,
                                    dsum=ws.dES if l == 0 else None)
            if l > 0 and self.sigma_tn_fused:
                with self._mark("tail_bwd_sigma_tn"):
                    ops.sigma_tn(do, ws.xt[l - 1], Sl, G[f"S{l + 1}"], ws.tn_slab, precision=self.edge_gemm)
            elif l > 0:
                # dS^{l+1} (edge part) = x_t^{l}^T do ; do^{l} = (do S^T) * x(1-x), written over x^{l}
                with self._mark("tail_dS_tn"):
                    ops.gemm_tn(ws.xt[l - 1], do, G[f"S{l + 1}"], ws.tn_slab, a_planes=pl, **pk)
                with self._mark("tail_bwd_gemm"):
                    ops.rowgemm(do, Sl, ws.xt[l - 1], b_trans=True, act=L.ACT_DSIGMOID, aux=ws.xt[l - 1],
                                planes=L.PLANES_AUX if pl else 0, precision=self.edge_gemm)
            if side is not None:
                torch.cuda.current_stream().wait_stream(side)
            # head side (node level)
            if fused:
                ops.head_dz(ws.Ssm[l], Wl, ed.hptr, ed.hperm, ws.dWedge, ws.dwh, ws.dz)
            else:
                ops.head_bwd_node(dOn, Pl, ws.Ssm[l], Wl, ws.dP, ws.dz, hseg_ptr=ed.hptr, hperm=ed.hperm,
                                  dWedge=ws.dWedge, dsum=ws.dES if l == 0 else None)
            Xin = ws.X[l - 1] if l > 0 else P["E"]
            ws.WaT.copy_(P[f"Wa{l + 1}"].t())
            ops.gemm_tn_narrow(Xin, ws.dz, G[f"Wa{l + 1}"], G[f"ba{l + 1}"], ws.narrow_slab)
            # node-level weight gradients of the layer, batched (one launch per L.TN_BATCH): the head-chain
            # part of dS (added to the edge part, layers 2-3) or dS1, and dK_r = AE_r^T dP_r
            K, dK = P[f"K{l + 1}"], G[f"K{l + 1}"]
            sh = self.node_shard
            tn = [(Xin, dOn, G[f"S{l + 1}"], True) if l > 0 else (P["E"], ws.dES, G["S1"], False)]
            if sh is None:
                tn += [(ws.AE[r], ws.dP[r], dK[r], False) for r in range(R)]
            for i in range(0, len(tn), L.TN_BATCH):
                ops.gemm_tn_batched(tn[i:i + L.TN_BATCH], ws.tn_slab, **pk)
            if l > 0:
                ops.rowgemm(dOn, Sl, dOn_next, b_trans=True, coef=ws.dz, V=ws.WaT, v_rel_stride=D,
                            v_row_stride=0, act=L.ACT_DSIGMOID, aux=Xin, **pr)
            else:
                # dE (head input of layer 1 + x·S1 inputs of both sides)
                ops.rowgemm(ws.dES, Sl, G["E"], b_trans=True, coef=ws.dz, V=ws.WaT, v_rel_stride=D,
                            v_row_stride=0, **pr)
            # relation kernels: dK_r = AE_r^T dP_r (above) ; dAE_r += dP_r K_r^T
            if sh is None:
                ops.rowgemm_batched([(ws.dP[r], K[r], ws.dAE[r], dict(b_trans=True, accumulate=(l != 2), **pn))
                                     for r in range(R)])
            else:
                # relation-sharded: the owners sum the edge partials of dP, then form their rows of dK_r (a
                # partial over rows, all-reduced with the other small gradients) and of dAE_r
                sh.reduce_scatter(ws.dP.view(R * N, D))
                dK.zero_()
                for r, n0, n1 in sh.pieces():
                    ops.gemm_tn(ws.AE[r][n0:n1], ws.dP[r][n0:n1], dK[r], ws.tn_slab, accumulate=True, **pk)
                ops.rowgemm_batched([(ws.dP[r][n0:n1], K[r], ws.dAE[r][n0:n1],
                                      dict(b_trans=True, accumulate=True, **pn)) for r, n0, n1 in sh.pieces()])
            dOn, dOn_next = dOn_next, dOn
        # DistMult rel grad and the loss: every gradient past E is final now
        ops.reduce_slabs(ws.drel_slab, ws.nb_dm, G["rel"])
        ops.reduce_slabs(ws.loss_slab, ws.nb_dm, G.loss)
        if comm is not None:
            comm.ready(G.buf[N * D:])
        # dE += sum_r A_r^T dAE_r  (gradient through all_e -> sparse_dense_matmul); per-row sums, so a
        # row-chunked launch sequence is bitwise the single launch
        bptr, bcol, bval = adj.bwd_ptr, adj.bwd_col, adj.bwd_val
        if self.spmm_shard is not None and self.node_shard is None:
            # the owners of dAE's (relation, row) range get its sums over the ranks; each rank's transposed
            # SpMM runs over the entries in its range only, and dE's all-reduce below adds the ranks' parts
            self.spmm_shard.reduce_scatter(ws.dAE.view(R * N, D))
            bptr, bcol, bval = adj.bwd_columns(self.spmm_shard.a, self.spmm_shard.b)
        chunks = comm.row_chunks(N) if comm is not None else [(0, N)]
        for n0, n1 in chunks:
            ops.spmm_csr(bptr[n0:n1 + 1], bcol, bval, ws.dAE.view(R * N, D),
                         G["E"][n0:n1].view(1, n1 - n0, D), 1, n1 - n0, accumulate=True)
            if comm is not None:
                comm.ready(G["E"][n0:n1].reshape(-1))

    # -- node-partitioned step (parallel.NodeShard) -------------------------------
    def _dm_seed(self, T):
        if self._pred_seed is None:        # Keras BCE, x 1/num_entities (IDDGCN.py:161-168)
            return 1.0 / (float(self._t_global or T) * float(self.N)), True
        return float(self._pred_seed), False

    _e_pending = None      # the asynchronous all-gather of E after an owner-row Adam (node-partitioned train_step)
    # node-partitioned train_step with E owned by rows: False (default) completes the all-gather of E before train_step
    # returns, so params are whole for any reader (to_numpy, a checkpoint, predict) or writer (load); True leaves it in
    # flight for the next forward to complete after its owner-local work (bench.py's timed loop) — until then the other
    # ranks' rows of params["E"] are stale and must be neither read nor written (finish_pending() completes it)
    overlap_e_gather = False
    # split E collectives (opt-in, round 6): with owner_e, E travels as one broadcast per owner
    # instead of one all-gather, and the next forward's A_r E runs as one SpMM per source owner, each after its piece
    # has landed (the own rows' first); dE is reduced to each owner as soon as the transposed SpMM has written that
    # owner's rows.  Results within fp32 reordering of the unsplit step (the per-row sums add the owners' partial
    # sums); bounded to ~2 ms per config-5 rank step by the SpMMs it can hide behind (Multi-GPU)
    split_e_collectives = False
    _e_parts = None

    def finish_pending(self):
        """Complete the all-gather of E a node-partitioned train_step left in flight (the next forward does it
        itself, after its owner-local work): every rank's E whole again."""
        pend, self._e_pending = self._e_pending, None
        if pend is not None:
            pend.wait()
        parts, self._e_parts = self._e_parts, None
        if parts is not None:
            for h in parts.values():
                h.wait()

    def _owner_csr(self, adj, sh):
        """The owned rows' forward CSR of every relation cut by the owner of the column (split E collectives): {(r, k):
        (row_ptr, col, val)} over rows [a, b), each row's entries of owner k in their original order."""
        # the adjacency itself is held beside the key (an id() could be reused by a later graph)
        key = (sh.a, sh.b, tuple(sh.cuts))
        if getattr(self, "_ocsr_adj", None) is adj and self._ocsr_key == key:
            return self._ocsr
        N, R = self.N, self.R
        a, b = sh.a, sh.b
        dev = adj.fwd_col.device
        inner = torch.tensor(sh.cuts[1:-1], dtype=torch.int64, device=dev)
        out = {}
        for r in range(R):
            ptr = adj.fwd_ptr[r * (N + 1) + a:r * (N + 1) + b + 1].long()
            p0, p1 = int(ptr[0]), int(ptr[-1])
            col = adj.fwd_col[p0:p1]
            val = adj.fwd_val[p0:p1] if adj.fwd_val is not None else None      # (None: every value 1)
            rows = torch.repeat_interleave(torch.arange(b - a, device=dev), ptr[1:] - ptr[:-1])
            own = torch.bucketize(col.long(), inner, right=True)
            for k in range(sh.world):
                m = own == k
                cnt = torch.bincount(rows[m], minlength=b - a)
                kp = torch.zeros(b - a + 1, dtype=torch.int64, device=dev)
                kp[1:] = torch.cumsum(cnt, 0)
                out[(r, k)] = (kp.int().contiguous(), col[m].contiguous(), None if val is None else val[m].contiguous())
        self._ocsr_adj, self._ocsr_key, self._ocsr = adj, key, out
        return out

    def _forward_rows(self, P, adj, ed, ws, train):
        """The forward with the node tables computed for the owned rows [a, b) only (parallel.NodeShard): the
        rank's scored edges all have their tail there, so the tail chain reads local P / ES1 rows; the edges'
        heads need W^l (all-gathered, N x R) and DistMult X^3 (all-gathered, N x D).  E S^1 and the layer-1 alpha
        read the owned E rows only: they run first, beside a pending all-gather of E (train_step's owner Adam)."""
        N, R, D, T = self.N, self.R, self.D, ed.T
        sh = self.row_shard
        a, b = sh.a, sh.b
        E = P["E"]
        pn = dict(precision=self.proj_gemm)
        pr = dict(precision=self.row_gemm)
        idx = sh.owned_idx(self.device)
        if b > a:
            ops.rowgemm(E[a:b], P["S1"], ws.ES1[a:b], **pn)
            ops.alpha_fwd(E[a:b], P["Wa1"], P["ba1"], ws.Ssm[0][a:b], ws.W[0][a:b])
        parts, self._e_parts = self._e_parts, None
        self.finish_pending()
        if b > a and parts is not None:
            # split E collectives: A_r E as one SpMM per source owner, the own rows first, each other owner's after
            # its broadcast has landed; the pieces add into the rows in that order
            ocsr = self._owner_csr(adj, sh)
            order = [sh.rank] + [k for k in range(sh.world) if k != sh.rank]
            for i, k in enumerate(order):
                if k != sh.rank:
                    parts[k].wait()
                for r in range(R):
                    kp, kc, kv = ocsr[(r, k)]
                    ops.spmm_csr(kp, kc, kv, E, ws.AE[r][a:b].view(1, b - a, D), 1, b - a, accumulate=i > 0)
        elif b > a:
            for r in range(R):              # A_r E over the owned rows (IDDGCN.py:69-70)
                ops.spmm_csr(adj.fwd_ptr[r * (N + 1) + a:r * (N + 1) + b + 1], adj.fwd_col, adj.fwd_val, E,
                             ws.AE[r][a:b].view(1, b - a, D), 1, b - a)
        if parts is not None:
            for h in parts.values():
                h.wait()
        if b > a:
            proj = [(ws.AE[r][a:b], P[f"K{l + 1}"][r], ws.P[l, r][a:b], pn) for l in range(NUM_LAYERS)
                    for r in range(R)]
            nb = L.ROWGEMM_BATCH
            for i in range(0, len(proj), nb):
                ops.rowgemm_batched(proj[i:i + nb])
        sh.all_gather(ws.W[0])
        # node level first (layers 1-3 over the owned rows, W^l all-gathered as each layer's alpha is known), so
        # that DistMult's head rows X^3 travel while ALL of the tail side runs (the layer-1 combine, the two tail
        # GEMMs: they read x^l, P^l, ES1 and the gathered W^l, and write x^l, nothing of X^3)
        if b > a:
            ops.combine(ws.ES1, ws.W[0][a:b], ws.P[0], ws.X[0][a:b], y_idx=idx, v_idx=idx)
        for l in (1, 2):
            if b > a:
                ops.alpha_fwd(ws.X[l - 1][a:b], P[f"Wa{l + 1}"], P[f"ba{l + 1}"], ws.Ssm[l][a:b], ws.W[l][a:b])
            sh.all_gather(ws.W[l])
            if b > a and R > 2 and D == 256 and ws.train:
                # as in forward(): the GEMM into a free N x D table (ES1 is still needed by the layer-1 tail combine
                # below; the head-seed buffer dOn_b is free until the backward), then the row-aligned combine
                tmp = ws.dOn_b[a:b]
                ops.rowgemm(ws.X[l - 1][a:b], P[f"S{l + 1}"], tmp, **pr)
                ops.combine(tmp, ws.W[l][a:b], ws.P[l], ws.X[l][a:b], v_idx=idx)
            elif b > a:
                ops.rowgemm(ws.X[l - 1][a:b], P[f"S{l + 1}"], ws.X[l][a:b], coef=ws.W[l][a:b], V=ws.P[l], v_idx=idx,
                            v_rel_stride=N * D, act=L.ACT_SIGMOID, **pr)
        x3 = sh.all_gather(ws.X[2], async_op=True)
        pl = self.use_planes
        ops.gather_rows(ws.W[0], ed.h, ws.Wedge[0])
        ops.combine(ws.ES1, ws.Wedge[0], ws.P[0], ws.xt[0], y_idx=ed.t, v_idx=ed.t, planes_out=pl)
        for l in (1, 2):
            ops.gather_rows(ws.W[l], ed.h, ws.Wedge[l])
            with self._mark("tail_fwd_gemm"):
                ops.rowgemm(ws.xt[l - 1], P[f"S{l + 1}"], ws.xt[l], coef=ws.Wedge[l], V=ws.P[l], v_idx=ed.t,
                            v_rel_stride=N * D, act=L.ACT_SIGMOID,
                            planes=(L.PLANES_A | (L.PLANES_C if l == 1 else 0)) if pl else 0, precision=self.edge_gemm)
        x3.wait()
        if train:
            scale, bce = self._dm_seed(T)
            ops.distmult_bce_heads(ed.hptr, ed.hperm, ws.X[2], ws.xt[2], ed.r, P["rel"], ed.y if bce else None,
                                   ws.xt[2], ws.dOn_a, ws.drel_slab, ws.loss_slab, scale=scale,
                                   p_out=ws.p if self._want_p else None, s_out=ws.s if self._want_p else None)
        else:
            ops.distmult_bce(ws.X[2], ed.h, ws.xt[2], ed.r, P["rel"], p_out=ws.p, s_out=ws.s)

    def _backward_rows(self, P, G, adj, ed, ws, comm, e_owner=False):
        """The backward of a node-partitioned step: the head seeds dO^3 and the dWedge head sums are
        reduce-scattered to the heads' owners, everything node-level runs over the owned rows, the tail
        segment sums are local; every gradient written is a partial over the rank's rows / edges, summed by
        ``comm`` (the flat gradient buffer's bucketed all-reduce).  ``e_owner``: dE is not all-reduced but
        reduce-scattered to the row owners (asynchronously; the handle is returned, and G["E"][a:b] holds the sums
        once it is waited for), for the owners' Adam (KerasAdam.apply_owned) and an all-gather of E."""
        N, R, D = self.N, self.R, self.D
        sh = self.row_shard
        a, b = sh.a, sh.b
        pk, pn, pr = dict(precision=self.gemm), dict(precision=self.proj_gemm), dict(precision=self.row_gemm)
        if getattr(ws, "ep", None) is None:
            ws.ep = torch.empty(N, R, dtype=torch.float32, device=self.device)
        dOn, dOn_next = ws.dOn_a, ws.dOn_b
        # head seeds dO^3 of the rank's edges -> the heads' owners, travelling while the layer-3 tail side runs (it
        # reads do^3, x^2, P^3, Wedge^3 and writes dP, dWedge, dS^3, do^2: nothing of dO^3)
        seeds = sh.reduce_scatter(dOn, async_op=True)
        pl = self.use_planes
        # the tail segments of the rank's edges are the owned rows' (edges are taken by tail): the tail reductions
        # run over [a, b) only, their dP / dES rows are the owned ones
        tptr = ed.tptr[a:b + 1]
        # bf16 edge tables at R = 8, D = 256 (config 5): layers 2 and 1 take the fused tail + head-term reduction (their
        # head seeds dO[a:b] are final: the node level of the layer above), then head_dz over the owned rows with the
        # reduce-scattered dWedge head sums; layer 3's head seeds are still on the wire during its tail reduction
        fuse = self.fuse_tail_head and self.features == "bf16" and R == 8 and D == 256
        for l in (2, 1, 0):
            Wl, Pl, Sl = ws.W[l], ws.P[l], P[f"S{l + 1}"]
            do = ws.xt[l]
            fused = fuse and l < 2
            if b > a and fused:
                ops.tail_seg_reduce_head(tptr, ws.Wedge[l], do, Pl[:, a:b], ws.dP[:, a:b], ws.dWedge, dOn[a:b],
                                         Wl[a:b], ws.dwh[a:b], dsum=ws.dES[a:b] if l == 0 else None)
            elif b > a:
                ops.tail_seg_reduce(tptr, None, ws.Wedge[l], do, Pl[:, a:b], ws.dP[:, a:b], ws.dWedge,
                                    dsum=ws.dES[a:b] if l == 0 else None)
            if l > 0 and self.sigma_tn_fused:
                with self._mark("tail_bwd_sigma_tn"):
                    ops.sigma_tn(do, ws.xt[l - 1], Sl, G[f"S{l + 1}"], ws.tn_slab, precision=self.edge_gemm)
            elif l > 0:
                with self._mark("tail_dS_tn"):
                    ops.gemm_tn(ws.xt[l - 1], do, G[f"S{l + 1}"], ws.tn_slab, a_planes=pl, **pk)
                with self._mark("tail_bwd_gemm"):
                    ops.rowgemm(do, Sl, ws.xt[l - 1], b_trans=True, act=L.ACT_DSIGMOID, aux=ws.xt[l - 1],
                                planes=L.PLANES_AUX if pl else 0, precision=self.edge_gemm)
            seeds.wait()
            ops.head_wsum(ed.hptr, ed.hperm, ws.dWedge, ws.ep)
            sh.reduce_scatter(ws.ep)             # dWedge head sums -> the heads' owners
            K, dK = P[f"K{l + 1}"], G[f"K{l + 1}"]
            Xin = ws.X[l - 1] if l > 0 else P["E"]
            ws.WaT.copy_(P[f"Wa{l + 1}"].t())
            if b > a:
                if fused:       # dW = dwh + the head sums: head_dz over one-entry "segments" n -> ep[a + n]
                    ops.head_dz(ws.Ssm[l][a:b], Wl[a:b], sh.owned_ptr(self.device), sh.owned_idx(self.device), ws.ep,
                                ws.dwh[a:b], ws.dz[a:b])
                else:
                    ops.head_bwd_node(dOn[a:b], Pl[:, a:b], ws.Ssm[l][a:b], Wl[a:b], ws.dP[:, a:b], ws.dz[a:b],
                                      ep=ws.ep[a:b], dsum=ws.dES[a:b] if l == 0 else None)
                ops.gemm_tn_narrow(Xin[a:b], ws.dz[a:b], G[f"Wa{l + 1}"], G[f"ba{l + 1}"], ws.narrow_slab)
                tn = [(Xin[a:b], dOn[a:b], G[f"S{l + 1}"], True) if l > 0 else (P["E"][a:b], ws.dES[a:b], G["S1"], False)]
                tn += [(ws.AE[r][a:b], ws.dP[r][a:b], dK[r], False) for r in range(R)]
                for i in range(0, len(tn), L.TN_BATCH):
                    ops.gemm_tn_batched(tn[i:i + L.TN_BATCH], ws.tn_slab, **pk)
                if l > 0:
                    ops.rowgemm(dOn[a:b], Sl, dOn_next[a:b], b_trans=True, coef=ws.dz[a:b], V=ws.WaT, v_rel_stride=D,
                                v_row_stride=0, act=L.ACT_DSIGMOID, aux=Xin[a:b], **pr)
                else:
                    ops.rowgemm(ws.dES[a:b], Sl, G["E"][a:b], b_trans=True, coef=ws.dz[a:b], V=ws.WaT,
                                v_rel_stride=D, v_row_stride=0, **pr)
                ops.rowgemm_batched([(ws.dP[r][a:b], K[r], ws.dAE[r][a:b],
                                      dict(b_trans=True, accumulate=(l != 2), **pn)) for r in range(R)])
            else:                                # an empty range: its partials are zero
                for k in (f"Wa{l + 1}", f"ba{l + 1}", f"K{l + 1}") + (("S1",) if l == 0 else ()):
                    G[k].zero_()
            dOn, dOn_next = dOn_next, dOn
        ops.reduce_slabs(ws.drel_slab, ws.nb_dm, G["rel"])
        ops.reduce_slabs(ws.loss_slab, ws.nb_dm, G.loss)
        if comm is not None:
            comm.ready(G.buf[N * D:])
        # dE: the owned rows' direct terms (above), zero elsewhere, + the transposed SpMM of the owned dAE rows
        G["E"][:a].zero_()
        G["E"][b:].zero_()
        bptr, bcol, bval = adj.bwd_node_rows(a, b)
        if e_owner and self.split_e_collectives:
            # split E collectives: the transposed SpMM by destination owner, each owner's dE rows reduced to it as soon
            # as they are written (owner order on every rank)
            hs = []
            for k in range(sh.world):
                n0, n1 = sh.cuts[k], sh.cuts[k + 1]
                if n1 > n0:
                    ops.spmm_csr(bptr[n0:n1 + 1], bcol, bval, ws.dAE.view(R * N, D),
                                 G["E"][n0:n1].view(1, n1 - n0, D), 1, n1 - n0, accumulate=True)
                hs.append(sh.reduce_rows(G["E"], k))
            from .parallel import _All
            return _All(hs)
        if e_owner:
            ops.spmm_csr(bptr, bcol, bval, ws.dAE.view(R * N, D), G["E"].view(1, N, D), 1, N, accumulate=True)
            return sh.reduce_scatter(G["E"], async_op=True)
        chunks = comm.row_chunks(N) if comm is not None else [(0, N)]
        for n0, n1 in chunks:
            ops.spmm_csr(bptr[n0:n1 + 1], bcol, bval, ws.dAE.view(R * N, D),
                         G["E"][n0:n1].view(1, n1 - n0, D), 1, n1 - n0, accumulate=True)
            if comm is not None:
                comm.ready(G["E"][n0:n1].reshape(-1))

    # -- public steps ---------------------------------------------------------
    def train_step(self, params, grads, opt, adj, ed, t_global=None, comm=None):
        """One full-batch step (IDDGCN.py:123-178).  Returns the device scalar (grads.loss) holding the
        sum of per-edge BCE terms (divide by the global T for the mean).  ``comm``: the data-parallel
        all-reduce (parallel.BucketedAllReduce), overlapped with the end of the backward."""
        ws = self.workspace(ed.T, True)
        self._t_global = t_global
        self.forward(params, adj, ed, ws, True)
        sh = self.row_shard
        if sh is not None and getattr(sh, "owner_e", False) and comm is not None:
            # node-partitioned step, E owned by rows (round 5): dE reduce-scattered to the owners, Adam over the owned
            # E rows only, E all-gathered asynchronously — the next forward runs its owner-local work (E S^1 and the
            # layer-1 alpha of the owned rows) before it waits (finish_pending)
            rs = self.backward(params, grads, adj, ed, ws, comm, e_owner=True)
            D = self.D
            opt.apply_owned(params, grads, comm, rs, sh.a * D, sh.b * D)
            if self.split_e_collectives:
                self._e_parts = sh.broadcast_rows(params["E"])
            else:
                self._e_pending = sh.all_gather(params["E"], async_op=True)
            if not self.overlap_e_gather:
                self.finish_pending()
            return grads.loss
        self.backward(params, grads, adj, ed, ws, comm)
        if comm is not None and hasattr(comm, "finish_each") and hasattr(opt, "apply_overlapped"):
            opt.apply_overlapped(params, grads, comm)
        else:
            if comm is not None:
                comm.finish()
            opt.apply(params, grads)
        return grads.loss

    def predict(self, params, adj, ed, logits=False):
        """Probabilities p = sigmoid(s) of the scored edges (caller's order); with ``logits=True``
        also the pre-sigmoid DistMult scores s (IDDGCN.py:108)."""
        self.finish_pending()
        ws = self.workspace(ed.T, False)
        self.forward(params, adj, ed, ws, False)
        return (ed.unsort(ws.p), ed.unsort(ws.s)) if logits else ed.unsort(ws.p)

    def layer_outputs(self, ed, rows=None):
        """After a predict() forward: the per-edge layer outputs (x_h^l, x_t^l), l = 1..3, of the
        reference's IDDGCN_Layer calls (IDDGCN.py:238-274), in the caller's edge order (optionally only
        the caller rows ``rows``): the head chain gathered from the node table X^l, the tail chain
        un-permuted from the tail-sorted edge table x^l."""
        ws = self.workspace(ed.T, False)
        inv = ed.inv if rows is None else ed.inv[torch.as_tensor(rows, device=ed.inv.device)]
        heads = ed.h.long()[inv]
        pl = self.use_planes
        return [(ws.X[l][heads], ops.planes_to_f32(ws.xt[l][inv]) if pl and l < 2 else ws.xt[l][inv].float())
                for l in range(NUM_LAYERS)]

    def loss_and_grads(self, params, grads, adj, ed, t_global=None, logits=False):
        """Forward + backward without the optimizer step: (loss sum, p) or, with ``logits=True``,
        (loss sum, p, s) — s the pre-sigmoid DistMult scores — all per edge in the caller's order."""
        self.finish_pending()
        ws = self.workspace(ed.T, True)
        self._t_global = t_global
        self._want_p = True
        try:
            self.forward(params, adj, ed, ws, True)
        finally:
            self._want_p = False
        self.backward(params, grads, adj, ed, ws)
        if logits:
            return grads.loss, ed.unsort(ws.p), ed.unsort(ws.s)
        return grads.loss, ed.unsort(ws.p)


    def value_grads(self, params, adj, ed, scale=1.0, grads=None):
        """Gradient of ``scale * sum_e p_e`` (p = the model's predicted probabilities of the scored
        edges ``ed``) w.r.t. every stored adjacency value, and p.

        This is ``tape.gradient(pred, adj_mat.values)`` of the explainers (explaiNE.py:85-94,
        GnnExplainer.py:31-51): AE_r = A_r·E enters every layer, so with dAE_r the total gradient
        w.r.t. AE_r (summed over the 3 layers by the backward), d/dA_r[i,j] = <dAE_r[i], E[j]>, one
        SDDMM over the adjacency.  Returns (list of per-relation GPU tensors in the adjacency's
        entry order, p in the caller's edge order).  ``grads``: optional FlatParams that receives
        the parameter gradients of the same quantity (a scratch buffer is used otherwise).
        """
        N, R, D = self.N, self.R, self.D
        ws = self.workspace(ed.T, True)
        if grads is None:
            if getattr(self, "_scratch_grads", None) is None:
                self._scratch_grads = FlatParams(N, R, D, self.device)
            grads = self._scratch_grads
        if self.node_shard is not None or self.spmm_shard is not None or self.row_shard is not None:
            # a sharded backward leaves only this rank's rows of dAE (or its reduce-scattered range): the
            # SDDMM below needs the full per-rank dAE
            raise L.IddgcnError("value_grads: not available on an Engine with node_shard / spmm_shard / row_shard set")
        self._pred_seed, self._want_p = float(scale), True
        try:
            self.forward(params, adj, ed, ws, True)
            self.backward(params, grads, adj, ed, ws)
        finally:
            self._pred_seed, self._want_p = None, False
        dv = torch.empty(adj.total_nnz, dtype=torch.float32, device=self.device)
        ops.sddmm_csr(adj.fwd_ptr, adj.fwd_col, ws.dAE, params["E"], dv, R, N)
        return adj.to_entry_order(dv), ed.unsort(ws.p)


def step_flops(N, R, D, T, M):
    """Algorithmic work of one training step (W_gemm)."""
    return 12 * D * D * T + 18 * (R + 1) * N * D * D + 4 * M * D


def step_bytes(N, R, D, T, M, L=NUM_LAYERS):
    """Algorithmic HBM bytes of one training step (Q_hbm, fp32)."""
    return 40 * T * D + 8 * L * R * T * D + 24 * T + 16 * M + 16 * L * (R + 1) * N * D


MALL_BYTES = 256 * 2 ** 20          # the Infinity Cache (MI355X_MICROARCH.md): a gathered table this small is read once
LINE = 128                          # bytes an HBM access moves for a row gathered in random order (an L2 line)


def step_bytes_impl(N, R, D, T, M, eb=4, fused_sigma_tn=True, fused_tail_head=False):
    """Compulsory HBM bytes and GEMM work of one training step of THIS formulation (round 6), part by part (one part =
    the launches of one Engine.forward / backward stage): every table a kernel needs read once and every table it
    produces written once, where

      * gathers of tail-sorted rows (P_r^l[t], ES1[t]) read each distinct node row once per kernel (the rows of a tail
        run are consecutive edges: the distinct-row count, not R rows per scored edge as SURVEY §8(d)'s 8·L·R·T·D);
      * the SpMMs' column gathers read the gathered table once if it fits the 256 MiB Infinity Cache, else one row per
        stored entry (E at configs 4 / 5 is 1 GB: 4·M·D per SpMM);
      * rows of fewer than 128 B gathered or scattered in random (head) order move one 128-B line each (W^l[h_e] into
        the per-edge table, the dWedge head sums), the HBM access granularity.

    eb: bytes per edge-table element (4 fp32, 2 in the bf16-feature mode).  fused_sigma_tn: the layer-2/3 dS TN and
    sigma' backward as one pass (do^l, x^{l-1} read once) rather than two.  fused_tail_head: the R = 8 bf16 tail
    reduction that adds the head chain's node terms (its head side reads only the dWedge head sums).
    Returns (total bytes, {part: (bytes, algorithmic GEMM flop, "edge" | "node" | None)}); the flop sum is SURVEY
    §8(d)'s W_gemm less the SpMMs.  bench.py step_roofline "impl" prices each part at the larger of its MFMA and HBM
    time (a lower bound of a step whose parts run one after another); the PMC step totals of profiles/r06 show how
    close the kernels come to the bytes."""
    f = 4.0
    NDf, RNDf, TDe = N * D * f, R * N * D * f, T * D * eb
    G = 2.0 * D * D                                                           # flop per row of a D x D GEMM
    small_row = lambda nbytes: max(float(nbytes), LINE)          # noqa: E731
    gath_E = NDf if NDf <= MALL_BYTES else M * D * f
    gath_dAE = RNDf if RNDf <= MALL_BYTES else M * D * f
    L_ = NUM_LAYERS
    p = {}
    # forward
    p["spmm_fwd"] = (4.0 * M + 4.0 * R * (N + 1) + gath_E + RNDf, 0.0, None)
    p["projections"] = (RNDf + NDf + (L_ * RNDf + NDf), (L_ * R + 1) * G * N, "node")   # AE_r, E -> P_r^l, ES1
    p["alpha"] = (L_ * (NDf + 2 * N * R * f), 0.0, None)
    p["gather_W"] = (L_ * (4.0 * T + T * small_row(R * f)), 0.0, None)               # h_e, W^l[h_e] -> Wedge
    p["head_chain"] = (L_ * (2 * NDf + RNDf + N * R * f), (L_ - 1) * G * N, "node")  # X^{l-1}|ES1, P^l, W^l -> X^l
    p["tail_l1_combine"] = (NDf + RNDf + T * R * f + 4.0 * T + TDe, 0.0, None)       # ES1[t], P^1[t], Wedge -> x^1
    p["tail_fwd_gemm"] = ((L_ - 1) * (2 * TDe + T * R * f + 4.0 * T + RNDf), (L_ - 1) * G * T, "edge")
    p["distmult"] = (NDf + 2 * TDe + 16.0 * T + NDf, 0.0, None)                      # X^3[h], x^3 -> do^3, dO^3
    # backward, per layer
    if fused_tail_head:     # do, Wedge, P[t], dO, W -> dP, dWedge, <dO, P>; head side: dWedge[hperm] -> dz
        p["tail_reduce"] = (L_ * (TDe + 2 * T * R * f + 2 * RNDf + NDf) + NDf, 0.0, None)
        p["head_bwd"] = (L_ * (4.0 * T + T * small_row(R * f)), 0.0, None)
    else:                   # do, Wedge, P[t] -> dP, dWedge (+dES); head side: dO, P, dP (rw), dWedge[hperm] -> dz
        p["tail_reduce"] = (L_ * (TDe + 2 * T * R * f + 2 * RNDf) + NDf, 0.0, None)
        p["head_bwd"] = (L_ * (NDf + 3 * RNDf + 4.0 * T + T * small_row(R * f)), 0.0, None)
    p["edge_sigma_tn"] = ((L_ - 1) * (3 * TDe if fused_sigma_tn else 5 * TDe), 2 * (L_ - 1) * G * T, "edge")
    p["node_tn"] = (L_ * (2 * NDf + 2 * RNDf + NDf + N * R * f), L_ * (R + 1) * G * N, "node")  # dS head, dK_r, dW_a
    p["head_chain_bwd"] = (L_ * 3 * NDf, L_ * G * N, "node")                        # dO, X (dES) -> dO' (dE)
    p["dAE"] = (L_ * 2 * RNDf + (L_ - 1) * RNDf, L_ * R * G * N, "node")             # dP (+ dAE) -> dAE
    p["spmm_bwd"] = (4.0 * M + 4.0 * R * (N + 1) + gath_dAE + 2 * NDf, 0.0, None)
    p["adam"] = (7 * NDf, 0.0, None)                                                 # E: var, m, v, g -> var, m, v
    return sum(v[0] for v in p.values()), p
