"""Config 5 at full size: the forward's logit error against the float64 oracle (on the same bf16-rounded tail tables,
tests/test_gpu_config5.py's comparison) for each operand form of the bf16 edge GEMMs — weights (and the R = 8
combine's node rows / coefficients) as bf16 hi + lo, weights rounded to bf16 with the combine kept hi + lo
(IDDGCN_GEMM_BF16), and every operand rounded (precision 5, an experiment form of the R = 8 forward kernel) — so the
error each rounding adds can be read beside the test's bars (logits 2e-2 max, 5e-3 on 99% of edges).

usage: python tools/cfg5_operand_error.py
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from iddgcn_amd import ops  # noqa: E402
from iddgcn_amd.engine import Engine, FlatParams  # noqa: E402
from iddgcn_amd.graph import get_adj_mats  # noqa: E402
from iddgcn_amd.sampling import negative_samples  # noqa: E402
from iddgcn_amd.utils import synthetic_graph  # noqa: E402
from oracle.ref_model import forward_detail  # noqa: E402
from oracle.ref_utils import get_adj_coo  # noqa: E402
from test_gpu_config5 import D, M, N, NEG_EVERY, R, mild_params  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    ops._PRECISION[5] = 5
    pos, _ = synthetic_graph(N, R, M, seed=0)
    neg = negative_samples(pos[::NEG_EVERY], N, 89, device=dev)
    tri = np.concatenate([pos, neg])
    lab = np.concatenate([np.ones(len(pos), np.float32), np.zeros(len(neg), np.float32)])
    eng = Engine(N, R, D, dev, gemm="split", features="bf16")
    adj = get_adj_mats(pos, N, R, device=dev)
    ed = eng.edges(tri, lab)
    sample = np.sort(np.random.default_rng(0).choice(len(tri), 10_000, replace=False))
    need = np.unique(np.concatenate([tri[sample, 0], tri[sample, 2]]))
    coo = get_adj_coo(pos[np.isin(pos[:, 0], need)], N, R)
    params = mild_params()
    P = FlatParams(N, R, D, dev)
    P.load(params)
    bf = lambda x: x.to(torch.bfloat16).to(x.dtype)  # noqa: E731
    _, s64, _ = forward_detail(params, tri[sample], coo, N, dtype=torch.float64, tail_round=bf)
    out = {}
    for name, prec in (("hilo", None), ("bf16 weights (IDDGCN_GEMM_BF16)", "bf16"), ("every operand bf16", 5)):
        Engine.edge_gemm = property(lambda self, p=prec: p if p is not None else self.row_gemm)
        _, s = eng.predict(P, adj, ed, logits=True)
        err = np.abs(s.cpu().numpy()[sample].astype(np.float64) - s64)
        out[name] = {"max": float(err.max()), "q99": float(np.quantile(err, 0.99)), "q50": float(np.median(err))}
        print(json.dumps({name: out[name]}), flush=True)
    print(json.dumps({"max_abs_logit": float(np.abs(s64).max())}))


if __name__ == "__main__":
    main()
