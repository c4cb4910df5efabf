"""Time and check the edge-level GEMM kernels alone at config-3 shape (T = 4M rows, D = 256, R = 2),
in the operand-precision modes (exact f32 MFMA, split-fp16 MFMA, bf16x3 MFMA).

For each case it prints the time per launch, the algorithmic TFLOP/s, and the max error of each
mode against an fp64 torch reference on the first `check` rows (absolute, over max |ref|).

usage: python tools/bench_gemm.py [T] [modes=exact,split,bf16x3] [lib.so ...]
  (each library is loaded in turn on the same inputs: build-flag variants of the same source)
"""
import os
import sys

import torch

sys.path.insert(0, ".")
from iddgcn_amd import _lib as L  # noqa: E402
from iddgcn_amd import ops  # noqa: E402


def run(T=4_000_000, N=100_000, D=256, R=2, reps=5, check=20_000, modes=("exact", "split"), libs=()):
    for lp in libs or [None]:
        if lp:
            L._lib = L.load(lp)
            print(f"--- {lp}", flush=True)
        run1(T, N, D, R, reps, check, modes)


def run1(T, N, D, R, reps, check, modes):
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    A = torch.rand(T, D, device=dev, generator=g)
    S = torch.randn(D, D, device=dev, generator=g)
    W = torch.rand(N, R, device=dev, generator=g)
    h_ = torch.randint(0, N, (T,), device=dev, generator=g)
    Wedge = W[h_].contiguous()             # per-edge coefficients, as the engine passes them
    P = torch.randn(R, N, D, device=dev, generator=g) * 4
    t = torch.sort(torch.randint(0, N, (T,), device=dev, generator=g)).values.int()
    h = h_.int()
    aux = torch.rand(T, D, device=dev, generator=g)
    # gradient-like rows: tiny, spanning 6 decades from row to row (exercises the running scales)
    dO = torch.randn(T, D, device=dev, generator=g) * 1e-12 * 10 ** (6 * torch.rand(T, 1, device=dev, generator=g) - 3)
    C = torch.empty(T, D, device=dev)
    slab = torch.empty(ops.tn_blocks(T, D) * D * D, device=dev)
    dS = torch.empty(D, D, device=dev)
    n = check
    Ad, Sd = A[:n].double(), S.double()
    refs = {
        "fwd_combine": torch.sigmoid(Ad @ Sd + sum(W.double()[h[:n].long(), r:r + 1] * P.double()[r][t[:n].long()]
                                                   for r in range(R))),
        "bwd_dsig": (dO[:n].double() @ Sd.t()) * aux[:n].double() * (1 - aux[:n].double()),
        "plain": Ad @ Sd,
    }
    tn_ref = A.double().t() @ dO.double()
    for mname in modes:
        cases = {
            "fwd_combine": lambda: ops.rowgemm(A, S, C, coef=Wedge, V=P, v_idx=t, v_rel_stride=N * D,
                                               act=L.ACT_SIGMOID, precision=mname),
            "bwd_dsig": lambda: ops.rowgemm(dO, S, C, b_trans=True, act=L.ACT_DSIGMOID, aux=aux, precision=mname),
            "plain": lambda: ops.rowgemm(A, S, C, precision=mname),
            "tn": lambda: ops.gemm_tn(A, dO, dS, slab, precision=mname),
        }
        only = os.environ.get("IDDGCN_GEMM_CASES")
        for name, fn in cases.items():
            if only and name not in only.split(","):
                continue
            fn()
            torch.cuda.synchronize()
            err = ""
            if name in refs:
                ref = refs[name]
                e = ((C[:n].double() - ref).abs().max() / ref.abs().max()).item()
                err = f" relerr={e:.2e}"
            elif name == "tn":
                e = ((dS.double() - tn_ref).abs().max() / tn_ref.abs().max()).item()
                err = f" relerr={e:.2e}"
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                fn()
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / reps
            print(f"{mname:5s} {name:12s} {ms:7.3f} ms  {2.0 * D * D * T / ms / 1e9:6.1f} TF{err}", flush=True)


if __name__ == "__main__":
    a = sys.argv[1:]
    run(T=int(a[0]) if a else 4_000_000, modes=tuple(a[1].split(",")) if len(a) > 1 else ("exact", "split"),
        libs=a[2:])
