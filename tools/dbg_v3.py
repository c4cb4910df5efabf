import sys, torch, numpy as np
sys.path.insert(0, '.')
from iddgcn_amd import _lib as L, ops
dev = torch.device('cuda', 0)
g = torch.Generator().manual_seed(43)
for (M, R, use_ci, use_vi) in [(32000, 2, False, False), (32000, 2, True, False), (32000, 2, False, True), (32000, 2, True, True), (32000, 1, False, True), (9000, 2, True, True)]:
    D, N = 256, 700
    A = torch.randn(M, D, generator=g).to(dev)
    S = (torch.randn(D, D, generator=g) / 16).to(dev)
    kw = dict(coef=torch.rand(N if use_ci else M, R, generator=g).to(dev),
              coef_idx=torch.randint(0, N, (M,), generator=g).int().to(dev) if use_ci else None,
              V=torch.randn(R, N if use_vi else M, D, generator=g).to(dev),
              v_idx=torch.randint(0, N, (M,), generator=g).int().to(dev) if use_vi else None,
              v_rel_stride=(N if use_vi else M) * D, act=L.ACT_NONE)
    out = []
    for path in (0, 1):
        old = L.lib().iddgcn_set_rowgemm_path(path)
        C = torch.zeros(M, D, device=dev)
        ops.rowgemm(A, S, C, **kw)
        torch.cuda.synchronize()
        out.append(C)
        L.lib().iddgcn_set_rowgemm_path(old)
    bad = (out[0] != out[1])
    rows = bad.any(1).nonzero().flatten()
    nt = (M + 31) // 32
    tpb = (nt + 255) // 256
    tiles = (rows // 32)
    within = (tiles % tpb)
    print(M, R, use_ci, use_vi, 'tpb', tpb, 'bad rows', rows.numel(), 'tile-in-block hist', torch.bincount(within, minlength=tpb).tolist() if rows.numel() else [],
          'row-in-tile hist', torch.bincount(rows % 32, minlength=32).tolist()[:32] if rows.numel() else [], 'maxdiff', (out[0]-out[1]).abs().max().item())
    if rows.numel():
        cols = bad[rows[0]].nonzero().flatten()
        print('   first bad row', rows[0].item(), 'cols', cols[:5].tolist(), '... n', cols.numel())
