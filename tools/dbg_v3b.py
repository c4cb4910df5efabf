import sys, torch
sys.path.insert(0, '.')
from iddgcn_amd import _lib as L, ops
dev = torch.device('cuda', 0)
g = torch.Generator().manual_seed(1)
M, D, N, R = 32 * 1024, 256, 4096, 2
A = torch.zeros(M, D, device=dev)
S = torch.zeros(D, D, device=dev)
n = torch.arange(N, dtype=torch.float32)
V = torch.stack([n[:, None].expand(N, D), n[:, None].expand(N, D) * 0 + 0.0]).contiguous().to(dev)  # V0[n] = n, V1 = 0
vi = torch.randint(0, N, (M,), generator=g).int().to(dev)
coef = torch.ones(M, R, device=dev)
C = torch.zeros(M, D, device=dev)
ops.rowgemm(A, S, C, coef=coef, V=V, v_idx=vi, v_rel_stride=N * D)
torch.cuda.synchronize()
used = C[:, 0].round().long().cpu()
exp = vi.long().cpu()
ok = used == exp
print('ok rows', int(ok.sum()), 'of', M)
nt = M // 32; tpb = (nt + 255) // 256
bad = (~ok).nonzero().flatten()[:10]
for e in bad.tolist():
    u = used[e].item()
    cand = (exp == u).nonzero().flatten().tolist()[:5]
    print('row', e, 'tile', e // 32, 'tile-in-block', (e // 32) % tpb, 'row-in-tile', e % 32, 'used idx', u, 'expected', exp[e].item(), 'rows having that idx', cand)
# also columns: are all columns the same?
print('col-consistent', bool((C == C[:, :1]).all()))
