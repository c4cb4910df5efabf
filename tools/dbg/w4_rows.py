"""Where do the full-width bf16x3 GEMM's rows differ from the b3 kernel's (debug probe)."""
import sys
import torch
sys.path.insert(0, ".")
from iddgcn_amd import ops  # noqa: E402
for M in (64, 128, 64 * 256, 64 * 256 * 3 + 17, 400_000):
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    A = torch.rand(M, 256, device=dev, generator=g)
    S = torch.randn(256, 256, device=dev, generator=g)
    C0 = torch.zeros(M, 256, device=dev)
    C1 = torch.zeros(M, 256, device=dev)
    ops.rowgemm(A, S, C0, precision="bf16x3")
    ops.rowgemm(A, S, C1, precision="bf16x3", b_planes=ops.bf16x3_weight_planes(S))
    torch.cuda.synchronize()
    bad = ((C1 - C0).abs() > 1e-3 * C0.abs().max()).any(1).nonzero().flatten().cpu()
    print(M, "bad rows", bad.numel(), "first", bad[:8].tolist(), "row%64", sorted(set((bad % 64).tolist()))[:16],
          "tile", sorted(set((bad // 64).tolist()))[:10], flush=True)
    if bad.numel():
        r = int(bad[0])
        badc = ((C1[r] - C0[r]).abs() > 1e-3 * C0.abs().max()).nonzero().flatten().cpu()
        print("   row", r, "bad cols", badc[:40].tolist(), flush=True)
