"""Explainer throughput on the GPU (fold 4, bundled weights, the reference's 288 test triples) next to
the explainer oracle (reference formulation, torch-CPU fp32) on a bounded sample.

usage: python tools/bench_explain.py [n_gnn]   -> one JSON line
"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from iddgcn_amd import explain as X  # noqa: E402
from iddgcn_amd import get_IDDGCN_Model  # noqa: E402


def main(n_gnn=60):
    g = lambda n: dict(np.load(os.path.join(ROOT, "tests", "golden", n)))  # noqa: E731
    d, ex, w = g("fold4_data.npz"), g("explain_fold4.npz"), g("weights_fold4.npz")
    test = ex["test_triples"]
    adjacency = np.concatenate([d["X_train"].astype(np.int64), test])
    model = get_IDDGCN_Model(845, 4, 64, 64, 123, None, 0, 4)
    model.load_weights(os.path.join(ROOT, "tests", "golden", "weights_fold4.npz"))
    X.explaine(model, adjacency, test[:4])                   # warm-up (device state, workspaces)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    X.explaine(model, adjacency, test)
    torch.cuda.synchronize()
    t_ne = time.perf_counter() - t0
    init = np.random.default_rng(123).standard_normal((845, 845)).astype(np.float32)
    X.gnn_explainer(model, adjacency, test[:2], init_value=init)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    X.gnn_explainer(model, adjacency, test[:n_gnn], init_value=init)
    torch.cuda.synchronize()
    t_gnn = time.perf_counter() - t0
    from oracle import ref_explain
    ns = 8
    t0 = time.perf_counter()
    ref_explain.explaine(w, adjacency, test[:ns], 845, 4, dtype=torch.float32)
    t_ref_ne = time.perf_counter() - t0
    t0 = time.perf_counter()
    ref_explain.mask_explainer(w, adjacency, test[:4], 845, 4, init, dtype=torch.float32)
    t_ref_gnn = time.perf_counter() - t0
    print(json.dumps({
        "explaine_triples_per_s": len(test) / t_ne, "explaine_ms_per_triple": t_ne / len(test) * 1e3,
        "gnnexplainer_triples_per_s": n_gnn / t_gnn, "gnnexplainer_ms_per_triple": t_gnn / n_gnn * 1e3,
        "cpu_oracle": {"explaine_ms_per_triple": t_ref_ne / ns * 1e3, "gnnexplainer_ms_per_triple": t_ref_gnn / 4 * 1e3,
                       "cores": torch.get_num_threads(), "kind": "port",
                       "sample": f"{ns} / 4 triples, oracle/ref_explain.py reference formulation, torch-CPU fp32"},
        "config": {"workload": "fold4 explanation (N=845, R=4, D=64, 288 test triples, train+test adjacency)"},
    }), flush=True)


if __name__ == "__main__":
    main(*(int(a) for a in sys.argv[1:2]))
