"""Diagnostic: tests/test_gpu_config5.py::test_config5_bf16_forward_vs_oracle_on_rounded_tables with the new R = 8
forward (fwd_gather8_bf16_kernel) and with the v3 kernel (forced by a coefficient table that is not 16-B aligned):
logit errors against the float64 oracle on the same 10k sample, plus the magnitudes of the layer inputs."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from iddgcn_amd import ops  # noqa: E402
from iddgcn_amd.engine import Engine, FlatParams  # noqa: E402
from iddgcn_amd.graph import get_adj_mats  # noqa: E402
from iddgcn_amd.sampling import negative_samples  # noqa: E402
from iddgcn_amd.utils import synthetic_graph  # noqa: E402
from oracle.ref_model import forward_detail  # noqa: E402
from oracle.ref_utils import get_adj_coo  # noqa: E402
from test_gpu_config5 import mild_params, N, R, M, D, NEG_EVERY  # noqa: E402

cuda = torch.device("cuda", 0)
pos, _ = synthetic_graph(N, R, M, seed=0)
neg = negative_samples(pos[::NEG_EVERY], N, 89, device=cuda)
tri = np.concatenate([pos, neg])
lab = np.concatenate([np.ones(len(pos), np.float32), np.zeros(len(neg), np.float32)])
eng = Engine(N, R, D, cuda, features="bf16")
adj = get_adj_mats(pos, N, R, device=cuda)
ed = eng.edges(tri, lab)
sample = np.sort(np.random.default_rng(0).choice(len(tri), 10_000, replace=False))
need = np.unique(np.concatenate([tri[sample, 0], tri[sample, 2]]))
coo = get_adj_coo(pos[np.isin(pos[:, 0], need)], N, R)
params = mild_params()
P = FlatParams(N, R, D, cuda)
P.load(params)
bf = lambda x: x.to(torch.bfloat16).to(x.dtype)  # noqa: E731
p64, s64, _ = forward_detail(params, tri[sample], coo, N, dtype=torch.float64, tail_round=bf)
_orig = ops.rowgemm


def unaligned(A, B, C, **kw):
    if kw.get("coef") is not None and A.dtype == torch.bfloat16 and kw["coef"].shape[-1] == 8:
        c = kw["coef"]
        buf = torch.empty(c.numel() + 1, device=c.device, dtype=c.dtype)
        cu = buf[1:].view_as(c)
        cu.copy_(c)
        kw = dict(kw, coef=cu)
    return _orig(A, B, C, **kw)


from iddgcn_amd import _lib as L  # noqa: E402
outs = {}
for name in ("new", "v3", "new2", "batch16"):
    ops.rowgemm = unaligned if name == "v3" else _orig
    L.ROWGEMM_BATCH = 16 if name == "batch16" else 25
    p, s = eng.predict(P, adj, ed, logits=True)
    ss = s.cpu().numpy()[sample].astype(np.float64)
    err = np.abs(ss - s64)
    ws = eng.workspace(ed.T, False)
    outs[name] = [x.float().cpu() for _, x in eng.layer_outputs(ed, rows=sample[:2000])]
    print(f"{name}: logits max err {err.max():.3e} 99% {np.quantile(err, 0.99):.3e}", flush=True)
    if name in ("new", "batch16"):
        for l in range(3):
            print(f"  layer {l + 1}: max|P| {ws.P[l].abs().max().item():.3e} max|Wedge| {ws.Wedge[l].abs().max().item():.3e}",
                  flush=True)
for l in range(3):
    a, b = outs["new"][l], outs["v3"][l]
    d = (a - b).abs()
    print(f"x_t^{l + 1} new vs v3: max diff {d.max().item():.3e}, rows differing {(d.amax(1) > 0).float().mean().item():.3f}, "
          f"mean |diff| {d.mean().item():.3e}; new vs new2 bitwise {torch.equal(a, outs['new2'][l])}", flush=True)
