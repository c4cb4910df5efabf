"""Debug probe for tail_seg_mfma8_kernel: error pattern of dP against float64 by node degree / column / relation."""
import sys
import torch
sys.path.insert(0, ".")
from iddgcn_amd import ops  # noqa: E402

dev = torch.device("cuda", 0)
g = torch.Generator().manual_seed(0)
R, D = 8, 256
for lens in ([5, 32, 33, 64, 70, 1, 0, 17], [40] * 6):
    N = len(lens)
    t = torch.repeat_interleave(torch.arange(N), torch.tensor(lens))
    T = len(t)
    tptr = torch.cat([torch.zeros(1, dtype=torch.long), torch.cumsum(torch.tensor(lens), 0)]).int().to(dev)
    W = torch.rand(T, R, generator=g).to(dev)
    P = torch.randn(R, N, D, generator=g).to(dev)
    dO = torch.randn(T, D, generator=g).to(torch.bfloat16).to(dev)
    dP, dWe = torch.full((R, N, D), 7.0, device=dev), torch.full((T, R), 7.0, device=dev)
    ops.tail_seg_reduce(tptr, None, W, dO, P, dP, dWe)
    ref = torch.zeros(R, N, D, dtype=torch.float64, device=dev)
    for r in range(R):
        ref[r].index_add_(0, t.to(dev), W.double()[:, r:r + 1] * dO.double())
    err = (dP.double() - ref).abs()
    print("lens", lens, "max err", err.max().item(), "max ref", ref.abs().max().item())
    for n in range(N):
        e = err[:, n, :]
        bad = (e > 1e-4 * max(ref.abs().max().item(), 1e-9))
        print(f"  node {n} len {lens[n]}: max err {e.max().item():.3e} bad cols {bad.any(0).nonzero().flatten()[:16].tolist()} bad rels {bad.any(1).nonzero().flatten().tolist()}")
    # compare to sum over a subset of edges: which edges are missing?
    n = max(range(N), key=lambda k: err[:, k].max().item())
    beg = int(tptr[n]); end = int(tptr[n + 1])
    r = int(err[:, n].max(1).values.argmax()); c = int(err[r, n].argmax())
    terms = (W.double()[beg:end, r] * dO.double()[beg:end, c]).cpu()
    print("  worst node", n, "rel", r, "col", c, "got", dP[r, n, c].item(), "ref", ref[r, n, c].item())
    diff = dP[r, n, c].item() - ref[r, n, c].item()
    close = [(k, terms[k].item()) for k in range(len(terms)) if abs(terms[k].item() + diff) < 1e-3 or abs(terms[k].item() - diff) < 1e-3]
    print("  single terms matching the difference:", close[:5])
