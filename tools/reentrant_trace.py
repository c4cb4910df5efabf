"""Find the first launch whose output differs when engines run concurrently (see tools/reentrant_probe.py).

Every ops.* call of the engine is wrapped: after it returns, the tensors it may have written (by name) are
cloned on the current stream.  One step alone, then the same step with other engines running concurrently on
their own streams / threads; the traces are compared call by call and the first differing call is printed.

usage: python tools/reentrant_trace.py mode other_mode[,other...] [reps]
"""
import sys
import threading

import numpy as np
import torch

sys.path.insert(0, ".")
from iddgcn_amd import ops  # noqa: E402
from iddgcn_amd import engine as E  # noqa: E402
from iddgcn_amd.engine import Engine, FlatParams  # noqa: E402
from iddgcn_amd.graph import get_adj_mats  # noqa: E402
from iddgcn_amd.utils import synthetic_graph  # noqa: E402
from tests.test_gpu_reentrant import _params  # noqa: E402

_local = threading.local()
OUTS = {"spmm_csr": (4,), "rowgemm": (2,), "rowgemm_batched": (), "gemm_tn": (2,), "gemm_tn_batched": (),
        "gemm_tn_narrow": (2, 3), "alpha_fwd": (3, 4), "gather_rows": (2,), "combine": (3,),
        "distmult_bce_heads": (), "tail_seg_reduce": (5, 6), "head_bwd_node": (4, 5), "reduce_slabs": (2,)}


def wrap(name, fn):
    def w(*a, **kw):
        tr = getattr(_local, "trace", None)
        if tr is not None and name in ("tail_seg_reduce", "head_bwd_node"):
            # every tensor argument as it is when the launch is queued (stream order: after all earlier launches)
            ins = [x.clone() for x in list(a) + list(kw.values()) if torch.is_tensor(x)]
            tr.append((name + ".inputs", ins))
        r = fn(*a, **kw)
        if tr is not None:
            outs = [a[i] for i in OUTS.get(name, ()) if i < len(a) and torch.is_tensor(a[i])]
            if name == "rowgemm_batched":
                outs = [c[2] for c in a[0]]
            if name == "gemm_tn_batched":
                outs = [c[2] for c in a[0]]
            if name == "distmult_bce_heads":
                outs = [a[7], a[8]]
            tr.append((name, [o.clone() for o in outs]))
        return r
    return w


for n in OUTS:
    f = getattr(ops, n)
    setattr(ops, n, wrap(n, f))
E.ops = ops


def main(mode, others, reps=3):
    cuda = torch.device("cuda", 0)
    N, R, D = 4000, 2, 256
    pos, neg = synthetic_graph(N, R, 40_000, seed=13)
    tri = np.concatenate([pos, neg])
    lab = np.concatenate([np.ones(len(pos)), np.zeros(len(neg))])
    jobs = {}
    for m in [mode] + others:
        eng = Engine(N, R, D, cuda, gemm=m.split("#")[0])
        P, G = FlatParams(N, R, D, cuda), FlatParams(N, R, D, cuda)
        P.load(_params(N, R, D, 3))
        jobs[m] = dict(eng=eng, P=P, G=G, adj=eng.adjacency(get_adj_mats(pos, N, R)), ed=eng.edges(tri, lab))

    def run(j, trace):
        _local.trace = [] if trace else None
        j["eng"].loss_and_grads(j["P"], j["G"], j["adj"], j["ed"])
        t, _local.trace = _local.trace, None
        return t

    for j in jobs.values():
        run(j, False)
    ref = run(jobs[mode], True)
    torch.cuda.synchronize()
    stop = threading.Event()

    def bg(m):
        st = torch.cuda.Stream(device=cuda)
        with torch.cuda.stream(st):
            while not stop.is_set():
                run(jobs[m], False)
                st.synchronize()

    ths = [threading.Thread(target=bg, args=(m,)) for m in others]
    for t in ths:
        t.start()
    st = torch.cuda.Stream(device=cuda)
    for rep in range(reps):
        with torch.cuda.stream(st):
            tr = run(jobs[mode], True)
        st.synchronize()
        first = None
        for k, ((n1, o1), (n2, o2)) in enumerate(zip(ref, tr)):
            diffs = []
            for i, (x, y) in enumerate(zip(o1, o2)):
                if not torch.equal(x, y):
                    nd = int((x != y).sum().item())
                    # which 64-B chunks / rows: positions of differing elements
                    idx = (x != y).flatten().nonzero().flatten()
                    xf, yf = x.flatten(), y.flatten()
                    vals = ", ".join(f"{j}: {xf[j].item():.9e} -> {yf[j].item():.9e}" for j in idx[:3].tolist())
                    diffs.append(f"[{i}] {nd}/{x.numel()} max {(x - y).abs().max().item():.2e} first idx "
                                 f"{idx[:6].tolist()} ({vals}); max|ref| {xf.abs().max().item():.2e}")
            if diffs:
                first = f"call {k} {n1}: " + "; ".join(diffs)
                break
        print(f"{mode} rep {rep}: {first or 'bitwise'}", flush=True)
        if first:
            print("   calls: " + " ".join(f"{k}:{n}" for k, (n, _) in enumerate(ref)), flush=True)
    stop.set()
    for t in ths:
        t.join()


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2].split(","), int(sys.argv[3]) if len(sys.argv) > 3 else 3)
