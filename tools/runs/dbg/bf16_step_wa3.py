"""Diagnostic: test_bf16_mode_step_tracks_fp32[8]'s gradients per parameter, fp32 engine vs bf16 mode with the new
R = 8 forward (fwd_gather8_bf16_kernel) vs bf16 mode on the v3 kernel (forced by a coefficient table that is not
16-B aligned, which the new kernel's dispatch refuses).  Prints max |g| and the max deviation per parameter."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from iddgcn_amd import ops  # noqa: E402
from iddgcn_amd.engine import Engine, FlatParams  # noqa: E402
from iddgcn_amd.graph import get_adj_mats  # noqa: E402
from iddgcn_amd.utils import synthetic_graph  # noqa: E402

D, R, N = 256, 8, 1500
cuda = torch.device("cuda", 0)
pos, neg = synthetic_graph(N, R, 16000, seed=40 + R)
tri = np.concatenate([pos, neg])
lab = np.concatenate([np.ones(len(pos)), np.zeros(len(neg))])
rng = np.random.default_rng(R)
params = {"E": rng.standard_normal((N, D)) / np.sqrt(D), "rel": rng.standard_normal((R, D))}
for l in (1, 2, 3):
    params.update({f"K{l}": rng.standard_normal((R, D, D)) / D, f"S{l}": rng.standard_normal((D, D)) / np.sqrt(D),
                   f"Wa{l}": rng.standard_normal((D, R)) / np.sqrt(D), f"ba{l}": rng.standard_normal(R) * 0.1})

_orig = ops.rowgemm


def unaligned_rowgemm(A, B, C, **kw):
    if kw.get("coef") is not None and A.dtype == torch.bfloat16 and kw["coef"].shape[-1] == 8:
        c = kw["coef"]
        buf = torch.empty(c.numel() + 1, device=c.device, dtype=c.dtype)
        cu = buf[1:].view_as(c)
        cu.copy_(c)
        kw = dict(kw, coef=cu)
    return _orig(A, B, C, **kw)


out = {}
for name in ("f32", "bf16", "bf16_v3"):
    ops.rowgemm = unaligned_rowgemm if name == "bf16_v3" else _orig
    import iddgcn_amd.engine as E
    E.ops.rowgemm = ops.rowgemm
    eng = Engine(N, R, D, cuda, features="f32" if name == "f32" else "bf16")
    P, G = FlatParams(N, R, D, cuda), FlatParams(N, R, D, cuda)
    P.load(params)
    adj = eng.adjacency(get_adj_mats(pos, N, R))
    ed = eng.edges(tri, lab)
    loss, p = eng.loss_and_grads(P, G, adj, ed)
    ws = eng.workspace(ed.T, True)
    x3 = ws.xt[2][:ed.T].float().cpu() if name != "f32" else None
    out[name] = (float(loss.item()), p.cpu().numpy(), G.to_numpy())
    print(name, "loss", out[name][0], flush=True)
(l32, p32, g32) = out["f32"]
for k, v in g32.items():
    row = [f"{k:5s} max|g32| {np.abs(v).max():.3e}"]
    for name in ("bf16", "bf16_v3"):
        row.append(f"{name}: max|g| {np.abs(out[name][2][k]).max():.3e} dev {np.abs(out[name][2][k] - v).max():.3e}")
    print("  ".join(row))
print("p dev", np.abs(out["bf16"][1] - p32).max(), np.abs(out["bf16_v3"][1] - p32).max(),
      "new vs v3", np.abs(out["bf16"][1] - out["bf16_v3"][1]).max())
