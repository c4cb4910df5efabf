"""Diagnostic: config 5's forward node projections through the engine with a ROWGEMM_BATCH = 25 build (one launch
for all 25) vs one call per entry on the same operands.  usage: python tools/dbg/batch25_engine.py lib.so"""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from iddgcn_amd import _lib as L  # noqa: E402
from iddgcn_amd import ops  # noqa: E402
from iddgcn_amd.engine import Engine, FlatParams  # noqa: E402
from iddgcn_amd.graph import get_adj_mats  # noqa: E402
from iddgcn_amd.sampling import negative_samples  # noqa: E402
from iddgcn_amd.utils import synthetic_graph  # noqa: E402
from test_gpu_config5 import mild_params, N, R, M, D, NEG_EVERY  # noqa: E402
from tools.bench_mem import load_lenient  # noqa: E402

L._lib = load_lenient(sys.argv[1])
L.ROWGEMM_BATCH = 25
cuda = torch.device("cuda", 0)
pos, _ = synthetic_graph(N, R, M, seed=0)
neg = negative_samples(pos[::NEG_EVERY], N, 89, device=cuda)
tri = np.concatenate([pos, neg])
lab = np.concatenate([np.ones(len(pos), np.float32), np.zeros(len(neg), np.float32)])
eng = Engine(N, R, D, cuda, features="bf16")
adj = get_adj_mats(pos, N, R, device=cuda)
ed = eng.edges(tri, lab)
P = FlatParams(N, R, D, cuda)
P.load(mild_params())
calls = []
_orig = ops.rowgemm_batched


def spy(c):
    calls.append([(a, b, C, dict(kw)) for a, b, C, kw in c])
    return _orig(c)


ops.rowgemm_batched = spy
eng.predict(P, adj, ed)
torch.cuda.synchronize()
for i, c in enumerate(calls):
    print(f"batched call {i}: {len(c)} entries, M {[x[2].shape[0] for x in c][:3]}..., kw {c[0][3]}", flush=True)
    if len(c) < 20:
        continue
    ws = eng.workspace(ed.T, False)
    for k, (a, b, C, kw) in enumerate(c):
        ref = torch.empty_like(C)
        ops.rowgemm(a, b, ref, **kw)
        same = torch.equal(ref, C)
        print(f"  entry {k:2d}: {'ok' if same else 'DIFFERS'}  max|C| {C.abs().max().item():.3e} max|ref| "
              f"{ref.abs().max().item():.3e}  A {a.data_ptr() % 256} B {b.data_ptr() % 256} C {C.data_ptr() % 256} "
              f"B contiguous {b.is_contiguous()}", flush=True)
