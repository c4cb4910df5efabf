"""Where the exact-mode logit error comes from (config 3, full size, reference-distribution init).

For each combination of the edge-level and node-level GEMM operand precision, on a 10k scored-edge sample:
the logits' per-edge report (tests/parity.py) and the per-layer tail / head outputs against the float64 and
fp32 oracles, plus the node tables the forward gathers (P_r^l = AE_r K_r^l and ES1 = E S^1, at the sampled
tails) against float64.  usage (GPU box): python tools/logit_error_probe.py > gpurun_out/probe.json
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from iddgcn_amd.engine import Engine, FlatParams  # noqa: E402
from iddgcn_amd.graph import get_adj_mats  # noqa: E402
from iddgcn_amd.utils import synthetic_graph  # noqa: E402
from oracle.ref_model import adj_to_torch, forward_detail, init_params  # noqa: E402
from oracle.ref_utils import get_adj_coo  # noqa: E402
from parity import logit_report  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    N, R, M, D = 100_000, 2, 2_000_000, 256
    pos, neg = synthetic_graph(N, R, M, seed=0)
    tri = np.concatenate([pos, neg])
    adj = get_adj_mats(pos, N, R, device=dev)
    eng = Engine(N, R, D, dev)
    ed = eng.edges(tri)
    sample = np.sort(np.random.default_rng(0).choice(len(tri), 10_000, replace=False))
    st = tri[sample]
    need = np.unique(np.concatenate([st[:, 0], st[:, 2]]))
    coo = get_adj_coo(pos[np.isin(pos[:, 0], need)], N, R)
    params = init_params(N, R, D, seed=89)
    p64, s64, l64 = forward_detail(params, st, coo, N, dtype=torch.float64)
    p32, s32, l32 = forward_detail(params, st, coo, N, dtype=torch.float32)
    # float64 node tables at the sampled tails
    tails = np.unique(st[:, 2])
    A = adj_to_torch(coo, N, torch.float64)
    E = torch.as_tensor(params["E"], dtype=torch.float64)
    AE = [torch.sparse.mm(A[r], E)[torch.as_tensor(tails)] for r in range(R)]
    P64 = {(l, r): (AE[r] @ torch.as_tensor(params[f"K{l + 1}"][r], dtype=torch.float64)).numpy()
           for l in range(3) for r in range(R)}
    ES64 = (E[torch.as_tensor(tails)] @ torch.as_tensor(params["S1"], dtype=torch.float64)).numpy()
    P = FlatParams(N, R, D, dev)
    P.load(params)
    out = {}
    for edge, node in (("exact", "exact"), ("exact", "exact4"), ("exact", "split"), ("split", "split")):
        eng.gemm, eng.proj_gemm = edge, node
        _, s = eng.predict(P, adj, ed, logits=True)
        ws = eng.workspace(ed.T, False)
        rec = {"logits": logit_report(s.cpu().numpy()[sample], s64, s32)}
        ti = torch.as_tensor(tails, device=dev)
        for (l, r), ref in P64.items():
            got = ws.P[l, r][ti].double().cpu().numpy()
            rec[f"P{l + 1}_{r}_max_abs_err"] = float(np.abs(got - ref).max())
            rec[f"P{l + 1}_{r}_max_abs"] = float(np.abs(ref).max())
        rec["ES1_max_abs_err"] = float(np.abs(ws.ES1[ti].double().cpu().numpy() - ES64).max())
        for l, (xh, xt) in enumerate(eng.layer_outputs(ed, rows=sample), 1):
            for side, ours in ((0, xh), (1, xt)):
                o = ours.cpu().numpy().astype(np.float64)
                nm = f"layer{l}_{'head' if side == 0 else 'tail'}"
                rec[nm] = {"vs_fp64": float(np.abs(o - l64[l - 1][side]).max()),
                           "vs_fp32": float(np.abs(o - l32[l - 1][side]).max()),
                           "fp32_drift": float(np.abs(l32[l - 1][side] - l64[l - 1][side]).max())}
        out[f"edge={edge},node={node}"] = rec
        print(f"edge={edge} node={node}: {rec['logits']}", file=sys.stderr, flush=True)
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
