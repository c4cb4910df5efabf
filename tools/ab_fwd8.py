"""A/B of the config-5 forward GEMM form (R = 8 gathered relations, bf16 edge tables, split mode, degree 50)
across variant builds of libiddgcn_hip.so, round-robin on the same inputs (HIP events).
usage: python tools/ab_fwd8.py lib1.so lib2.so ... [--T 20000000 --N 400000]"""
import sys

import torch

sys.path.insert(0, ".")
from iddgcn_amd import _lib as L  # noqa: E402
from iddgcn_amd import ops  # noqa: E402
from tools.bench_mem import load_lenient, timeit  # noqa: E402


def main(libs, T=20_000_000, N=400_000, D=256, R=8, rounds=3):
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    A = torch.rand(T, D, device=dev, generator=g).bfloat16()
    C = torch.empty(T, D, device=dev, dtype=torch.bfloat16)
    S = torch.randn(D, D, device=dev, generator=g) / 16
    W = torch.rand(T, R, device=dev, generator=g)
    P = torch.randn(R, N, D, device=dev, generator=g)
    t = torch.sort(torch.randint(0, N, (T,), device=dev, generator=g)).values.int()
    for _ in range(rounds):
        for lib in libs:
            L._lib = load_lenient(lib)
            L._lib.iddgcn_set_gemm_precision(L.GEMM_SPLIT_F16)
            ms = timeit(lambda: ops.rowgemm(A, S, C, coef=W, V=P, v_idx=t, v_rel_stride=N * D, act=L.ACT_SIGMOID))
            print(f"{lib:24s} fwd8 T={T} N={N}: {ms:.3f} ms", flush=True)


if __name__ == "__main__":
    main([a for a in sys.argv[1:] if a.endswith(".so")])
