"""Is one node-level GEMM launch bitwise reproducible while other kernels run beside it on another stream?

Main stream: dK = AE^T dP (ops.gemm_tn, D = 256, M = N rows) and dAE = dP K^T (ops.rowgemm, plain, b_trans,
exact4 precision) over fixed random inputs, repeated; each result is compared bitwise with the one computed
with the GPU otherwise idle.  A second host thread keeps another stream busy with a chosen background
(a bf16x3 / exact edge-sized row GEMM, a copy) for the whole loop.

usage: python tools/concurrency_kernel_probe.py [background=b3|exact|copy|none] [reps] [N] [prec]
"""
import sys
import threading
import time

import torch

sys.path.insert(0, ".")
from iddgcn_amd import ops  # noqa: E402


def main(bg="b3", reps=50, N=4000, prec="exact"):
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    D = 256
    AE = torch.randn(N, D, device=dev, generator=g)
    dP = torch.randn(N, D, device=dev, generator=g) * 1e-3
    K = torch.randn(D, D, device=dev, generator=g) / 16
    slab = torch.empty(ops.tn_blocks(N, D) * D * D, device=dev)
    dK, dAE = torch.empty(D, D, device=dev), torch.empty(N, D, device=dev)

    def step():
        ops.gemm_tn(AE, dP, dK, slab, precision=prec)
        ops.rowgemm(dP, K, dAE, b_trans=True, precision="exact4" if prec == "exact" else prec)

    step()
    torch.cuda.synchronize()
    ref_k, ref_a = dK.clone(), dAE.clone()
    stop = threading.Event()

    def background():
        st = torch.cuda.Stream(device=dev)
        with torch.cuda.stream(st):
            T = 2_000_000
            A = torch.rand(T, D, device=dev)
            S = torch.randn(D, D, device=dev)
            C = torch.empty(T, D, device=dev)
            while not stop.is_set():
                if bg == "b3":
                    ops.rowgemm(A, S, C, precision="bf16x3")
                elif bg == "exact":
                    ops.rowgemm(A, S, C, precision="exact")
                elif bg == "copy":
                    C.copy_(A)
                st.synchronize()

    th = None
    if bg != "none":
        th = threading.Thread(target=background)
        th.start()
        time.sleep(1.0)
    bad_k = bad_a = 0
    worst_k = worst_a = 0.0
    st = torch.cuda.Stream(device=dev)
    with torch.cuda.stream(st):
        for _ in range(reps):
            step()
            st.synchronize()
            if not torch.equal(dK, ref_k):
                bad_k += 1
                worst_k = max(worst_k, (dK - ref_k).abs().max().item())
            if not torch.equal(dAE, ref_a):
                bad_a += 1
                worst_a = max(worst_a, (dAE - ref_a).abs().max().item())
    stop.set()
    if th is not None:
        th.join()
    print(f"bg={bg} prec={prec} N={N}: dK (TN) differs in {bad_k}/{reps} (max {worst_k:.2e}); "
          f"dAE (row GEMM) differs in {bad_a}/{reps} (max {worst_a:.2e})", flush=True)


if __name__ == "__main__":
    a = sys.argv[1:]
    main(a[0] if a else "b3", int(a[1]) if len(a) > 1 else 50, int(a[2]) if len(a) > 2 else 4000,
         a[3] if len(a) > 3 else "exact")
