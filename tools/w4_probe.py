"""A/B of the full-width bf16x3 row GEMM (w4, b_planes given) against the column-half kernel (b3) on identical
inputs at config-3 shape: time per launch (HIP events, median of rounds), error against float64 on sampled rows,
max |w4 - b3|, and a ragged M (rows past M untouched).

usage: python tools/w4_probe.py [--T 4000000] [--rounds 3] [--cases plain,fwd_combine,bwd_dsig,acc,bc]
"""
import argparse
import statistics
import sys

import torch

sys.path.insert(0, ".")
from iddgcn_amd import _lib as L  # noqa: E402
from iddgcn_amd import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", type=int, default=4_000_000)
    ap.add_argument("--N", type=int, default=100_000)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--cases", default="plain,fwd_combine,bwd_dsig,acc,bc")
    a = ap.parse_args()
    T, N, D, R = a.T, a.N, 256, 2
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    A = torch.rand(T, D, device=dev, generator=g)
    S = torch.randn(D, D, device=dev, generator=g)
    W = torch.rand(N, R, device=dev, generator=g)
    h = torch.randint(0, N, (T,), device=dev, generator=g)
    Wedge = W[h].contiguous()
    P = torch.randn(R, N, D, device=dev, generator=g) * 4
    t = torch.sort(torch.randint(0, N, (T,), device=dev, generator=g)).values.int()
    aux = torch.rand(T, D, device=dev, generator=g)
    dO = torch.randn(T, D, device=dev, generator=g) * 1e-3
    C0 = torch.randn(T, D, device=dev, generator=g)
    dz = torch.randn(T, R, device=dev, generator=g)
    WaT = torch.randn(R, D, device=dev, generator=g)
    pl = {False: ops.bf16x3_weight_planes(S, False), True: ops.bf16x3_weight_planes(S, True)}
    C = torch.empty(T, D, device=dev)
    rows = torch.cat([torch.arange(0, 2000, device=dev), torch.randint(0, T, (6000,), device=dev, generator=g),
                      torch.arange(T - 2000, T, device=dev)])
    Sd = S.double()

    def ref(name):
        if name == "plain":
            return A[rows].double() @ Sd
        if name == "fwd_combine":
            v = A[rows].double() @ Sd
            for r in range(R):
                v = v + Wedge[rows, r:r + 1].double() * P[r].double()[t[rows].long()]
            return torch.sigmoid(v)
        if name == "bwd_dsig":
            x = aux[rows].double()
            return (dO[rows].double() @ Sd.t()) * x * (1 - x)
        if name == "acc":
            return C0[rows].double() + A[rows].double() @ Sd.t()
        if name == "bc":
            x = aux[rows].double()
            v = dO[rows].double() @ Sd.t() + dz[rows].double() @ WaT.double()
            return v * x * (1 - x)

    def call(name, planes):
        def kw(bt):
            return dict(precision="bf16x3", b_planes=pl[bt] if planes else None)
        if name == "plain":
            return lambda: ops.rowgemm(A, S, C, **kw(False))
        if name == "fwd_combine":
            return lambda: ops.rowgemm(A, S, C, coef=Wedge, V=P, v_idx=t, v_rel_stride=N * D, act=L.ACT_SIGMOID,
                                       **kw(False))
        if name == "bwd_dsig":
            return lambda: ops.rowgemm(dO, S, C, b_trans=True, act=L.ACT_DSIGMOID, aux=aux, **kw(True))
        if name == "acc":
            return lambda: (C.copy_(C0), ops.rowgemm(A, S, C, accumulate=True, b_trans=True, **kw(True)))
        if name == "bc":
            return lambda: ops.rowgemm(dO, S, C, b_trans=True, coef=dz, V=WaT, v_rel_stride=D, v_row_stride=0,
                                       act=L.ACT_DSIGMOID, aux=aux, **kw(True))

    for name in a.cases.split(","):
        kid = {p: ops.rowgemm_kernel_id(A, S, C, precision="bf16x3", b_planes=pl[False] if p else None,
                                        **({} if name == "plain" else {"accumulate": name == "acc"}))
               for p in (False, True)} if name in ("plain", "acc") else {}
        outs, times = {}, {False: [], True: []}
        for p in (False, True):
            call(name, p)()
            torch.cuda.synchronize()
            outs[p] = C.clone()
        for _ in range(a.rounds):
            for p in (False, True):
                fn = call(name, p)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.reps):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                times[p].append(e0.elapsed_time(e1) / a.reps)
        rf = ref(name)
        errs = {p: ((outs[p][rows].double() - rf).abs().max() / rf.abs().max()).item() for p in (False, True)}
        diff = (outs[True] - outs[False]).abs().max().item()
        ms = {p: statistics.median(times[p]) for p in (False, True)}
        hw = 6 * 2.0 * D * D * T
        print(f"{name:12s} b3 {ms[False]:6.3f} ms ({hw / ms[False] / 1e9:6.1f} hwTF, err {errs[False]:.2e})  "
              f"w4 {ms[True]:6.3f} ms ({hw / ms[True] / 1e9:6.1f} hwTF, err {errs[True]:.2e})  max|w4-b3| {diff:.2e}"
              f"  ids {kid}  runs b3 {['%.3f' % x for x in times[False]]} w4 {['%.3f' % x for x in times[True]]}",
              flush=True)
    # ragged M: rows past M untouched
    M = T - 37
    C.fill_(7.0)
    ops.rowgemm(A, S, C[:M], precision="bf16x3", b_planes=pl[False])
    torch.cuda.synchronize()
    tail_ok = bool((C[M:] == 7.0).all().item())
    e = ((C[M - 100:M].double() - A[M - 100:M].double() @ Sd).abs().max()).item()
    print(f"ragged M={M}: rows past M untouched {tail_ok}, last rows abs err {e:.2e}", flush=True)


if __name__ == "__main__":
    main()
