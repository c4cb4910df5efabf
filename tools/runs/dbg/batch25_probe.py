"""Diagnostic: a 25-entry batched row GEMM (a build with ROWGEMM_BATCH = 25) at M rows per entry, laid out as
config 5's forward projections (entry l*8 + r reads A_r, plus E S^1), against one call per entry.
usage: python tools/dbg/batch25_probe.py lib.so M [precision] [busy]"""
import sys

import torch

sys.path.insert(0, ".")
from iddgcn_amd import _lib as L  # noqa: E402
from iddgcn_amd import ops  # noqa: E402
from tools.bench_mem import load_lenient  # noqa: E402

lib, M = sys.argv[1], int(sys.argv[2])
prec = sys.argv[3] if len(sys.argv) > 3 else "split"
L._lib = load_lenient(lib)
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(1)
D, R = 256, 8
A = [torch.randn(M, D, device=dev, generator=g) for _ in range(R + 1)]
Bs = [torch.randn(D, D, device=dev, generator=g) / 16 for _ in range(3 * R + 1)]
calls = [(A[r], Bs[l * R + r]) for l in range(3) for r in range(R)] + [(A[R], Bs[3 * R])]
outs = [torch.full((M, D), float("nan"), device=dev) for _ in calls]
busy = len(sys.argv) > 4 and sys.argv[4] == "busy"
ops.rowgemm_batched([(a, b, C, dict(precision=prec)) for (a, b), C in zip(calls, outs)])
if busy:             # many launches queued behind the batched one before anything waits for it
    x = torch.zeros(1024, device=dev)
    for _ in range(3000):
        x.add_(1.0)
torch.cuda.synchronize()
bad = []
for k, ((a, b), C) in enumerate(zip(calls, outs)):
    ref = torch.empty(M, D, device=dev)
    ops.rowgemm(a, b, ref, precision=prec)
    if not torch.equal(ref, C):
        bad.append((k, C.isnan().float().mean().item(), (C == 0).float().mean().item()))
print(f"M={M} {prec} busy={busy}: entries differing from single calls: {bad if bad else 'none'}", flush=True)
