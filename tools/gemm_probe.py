"""Run one edge-GEMM case a few times at config-3 shape (for rocprofv3 --pmc passes).

usage: python tools/gemm_probe.py {fwd,bwd,plain,tn,fwd8} {split,exact} [reps]
fwd8: the config-5 form (R = 8 relations, bf16 edge tables, degree 50) at T = 10M, N = 200k
"""
import sys

import torch

sys.path.insert(0, ".")
from iddgcn_amd import _lib as L  # noqa: E402
from iddgcn_amd import ops  # noqa: E402


def main(case, mode, reps=3, T=4_000_000, N=100_000, D=256, R=2):
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    if case == "fwd8":
        T, N, R = 10_000_000, 200_000, 8
    A = torch.rand(T, D, device=dev, generator=g)
    S = torch.randn(D, D, device=dev, generator=g)
    C = torch.empty(T, D, device=dev)
    if case == "fwd8":
        A = A.bfloat16()
        C = C.bfloat16()
        W = torch.rand(T, R, device=dev, generator=g)
        P = torch.randn(R, N, D, device=dev, generator=g)
        t = torch.sort(torch.randint(0, N, (T,), device=dev, generator=g)).values.int()
        fn = lambda: ops.rowgemm(A, S, C, coef=W, V=P, v_idx=t, v_rel_stride=N * D, act=L.ACT_SIGMOID, precision=mode)  # noqa
    elif case == "fwd":
        W = torch.rand(T, R, device=dev, generator=g)
        P = torch.randn(R, N, D, device=dev, generator=g)
        t = torch.sort(torch.randint(0, N, (T,), device=dev, generator=g)).values.int()
        fn = lambda: ops.rowgemm(A, S, C, coef=W, V=P, v_idx=t, v_rel_stride=N * D, act=L.ACT_SIGMOID, precision=mode)  # noqa
    elif case == "bwd":
        aux = torch.rand(T, D, device=dev, generator=g)
        fn = lambda: ops.rowgemm(A, S, C, b_trans=True, act=L.ACT_DSIGMOID, aux=aux, precision=mode)  # noqa
    elif case == "plain":
        fn = lambda: ops.rowgemm(A, S, C, precision=mode)  # noqa
    else:
        B = torch.randn(T, D, device=dev, generator=g)
        slab = torch.empty(ops.tn_blocks(T, D) * D * D, device=dev)
        dS = torch.empty(D, D, device=dev)
        fn = lambda: ops.gemm_tn(A, B, dS, slab, precision=mode)  # noqa
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    print(f"{case} {mode}: {ms:.3f} ms per launch, {2.0 * D * D * T / ms / 1e9:.1f} TFLOP/s algorithmic", flush=True)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 3)
