"""Debug probe 2: per source row, which columns the MFMA tail kernel gets wrong and where the value came from."""
import sys
import torch
sys.path.insert(0, ".")
from iddgcn_amd import ops  # noqa: E402

dev = torch.device("cuda", 0)
g = torch.Generator().manual_seed(0)
R, D, T = 8, 256, 32
tptr = torch.tensor([0, T], dtype=torch.int32).to(dev)
P = torch.randn(R, 1, D, generator=g).to(dev)
dO = torch.randn(T, D, generator=g).to(torch.bfloat16).to(dev)
dOf = dO.float().cpu()
for e in range(T):
    W = torch.zeros(T, R)
    W[e, :] = 1.0
    W = W.to(dev)
    dP, dWe = torch.full((R, 1, D), 7.0, device=dev), torch.full((T, R), 7.0, device=dev)
    ops.tail_seg_reduce(tptr, None, W, dO, P, dP, dWe)
    got = dP[0, 0].cpu()
    bad = (got != dOf[e]).nonzero().flatten().tolist()
    src = []
    for c in bad[:3]:
        w = (dOf == got[c]).nonzero().tolist()
        src.append((c, w[:2]))
    print(f"row {e}: {len(bad)} bad cols {bad[:4]}..{bad[-2:] if bad else ''} src {src}")
