"""Time the edge-level GEMM kernels alone at config-3 shape (T = 4M rows, D = 256, R = 2).

usage: python tools/bench_gemm.py [libpath ...]   (each lib is loaded in turn, same inputs)
"""
import ctypes
import sys

import torch

sys.path.insert(0, ".")
from iddgcn_amd import _lib as L  # noqa: E402
from iddgcn_amd import ops  # noqa: E402


def run(libpath, T=4_000_000, N=100_000, D=256, R=2, reps=5):
    L._lib = L.load(libpath)
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    A = torch.rand(T, D, device=dev, generator=g)
    S = torch.randn(D, D, device=dev, generator=g) / 16
    W = torch.rand(N, R, device=dev, generator=g)
    P = torch.randn(R, N, D, device=dev, generator=g)
    t = torch.sort(torch.randint(0, N, (T,), device=dev, generator=g)).values.int()
    h = torch.randint(0, N, (T,), device=dev, generator=g).int()
    aux = torch.rand(T, D, device=dev, generator=g)
    C = torch.empty(T, D, device=dev)
    slab = torch.empty(ops.tn_blocks(T, D) * D * D, device=dev)
    dS = torch.empty(D, D, device=dev)
    cases = {
        "fwd_combine": lambda: ops.rowgemm(A, S, C, coef=W, coef_idx=h, V=P, v_idx=t, v_rel_stride=N * D,
                                           act=L.ACT_SIGMOID),
        "bwd_dsig": lambda: ops.rowgemm(A, S, C, b_trans=True, act=L.ACT_DSIGMOID, aux=aux),
        "plain": lambda: ops.rowgemm(A, S, C),
        "tn": lambda: ops.gemm_tn(A, aux, dS, slab),
    }
    out = {}
    for name, fn in cases.items():
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        out[name] = (ms, 2.0 * D * D * T / ms / 1e9)
    print(libpath.split("/")[-1], " ".join(f"{k}={v[0]:.3f}ms/{v[1]:.1f}TF" for k, v in out.items()), flush=True)


if __name__ == "__main__":
    for p in sys.argv[1:] or [L.LIB_PATH]:
        run(p)
