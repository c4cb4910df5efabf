"""A/B of the node-level TN launches of one config-3 layer (three C = A^T B over N = 100k rows, D = 256, bf16x3:
the head chain's dS part and dK_r for R = 2) through ops.gemm_tn_batched, across library builds; results compared
with the first build's (max relative difference: a batched launch splits the rows differently) and with fp64.

usage: python tools/ab_tn_batched.py lib1.so [lib2.so ...]
"""
import sys

import torch

sys.path.insert(0, ".")
from iddgcn_amd import _lib as L  # noqa: E402
from iddgcn_amd import ops  # noqa: E402
from tools.bench_mem import load_lenient, timeit  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    N, D = 100_000, 256
    ents = [(torch.rand(N, D, device=dev, generator=g), torch.randn(N, D, device=dev, generator=g) * 1e-3,
             torch.empty(D, D, device=dev), k > 0) for k in range(3)]
    refs = [a.double().t() @ b.double() for a, b, _, _ in ents]
    slab = torch.empty(256 * D * D, device=dev)
    first = None
    for rnd in range(3):
        for p in sys.argv[1:]:
            L._lib = load_lenient(p)
            for _, _, c, _ in ents:
                c.zero_()
            ms = timeit(lambda: ops.gemm_tn_batched(ents, slab, precision="bf16x3"), reps=20)
            for _, _, c, _ in ents:
                c.zero_()
            ops.gemm_tn_batched([(a, b, c, False) for a, b, c, _ in ents], slab, precision="bf16x3")
            torch.cuda.synchronize()
            outs = [c.clone() for _, _, c, _ in ents]
            err = max(((o.double() - r).abs().max() / r.abs().max()).item() for o, r in zip(outs, refs))
            first = first or outs
            d = max(((o - f).abs().max() / f.abs().max()).item() for o, f in zip(outs, first))
            print(f"round {rnd} {p.split('/')[-1]:22s} {ms * 1e3:8.1f} us per 3-entry call  err vs fp64 {err:.2e}  "
                  f"vs first build {d:.2e}", flush=True)


if __name__ == "__main__":
    main()
