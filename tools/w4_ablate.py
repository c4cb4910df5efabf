"""Time the full-width bf16x3 plain row GEMM (w4) across library builds (ablation variants) on identical inputs,
the libraries alternating `rounds` times.  usage: python tools/w4_ablate.py [--T 4000000] [--case plain] lib.so ..."""
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
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--case", default="plain")
    ap.add_argument("libs", nargs="+")
    a = ap.parse_args()
    T, D, N, R = a.T, 256, 100_000, 2
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    A = torch.rand(T, D, device=dev, generator=g)
    S = torch.randn(D, D, device=dev, generator=g)
    C = torch.empty(T, D, device=dev)
    W = torch.rand(T, R, device=dev, generator=g)
    P = torch.randn(R, N, D, device=dev, generator=g)
    t = torch.sort(torch.randint(0, N, (T,), device=dev, generator=g)).values.int()
    aux = torch.rand(T, D, device=dev, generator=g)
    libs = {p: L.load(p) for p in a.libs}
    times = {p: [] for p in a.libs}
    ref = None
    for _ in range(a.rounds):
        for p in a.libs:
            L._lib = libs[p]
            bt = a.case == "bwd"
            pl = ops.bf16x3_weight_planes(S, bt)
            if a.case == "plain":
                fn = lambda: ops.rowgemm(A, S, C, precision="bf16x3", b_planes=pl)  # noqa
            elif a.case == "fwd":
                fn = lambda: ops.rowgemm(A, S, C, coef=W, V=P, v_idx=t, v_rel_stride=N * D, act=L.ACT_SIGMOID,  # noqa
                                         precision="bf16x3", b_planes=pl)
            else:
                fn = lambda: ops.rowgemm(A, S, C, b_trans=True, act=L.ACT_DSIGMOID, aux=aux, precision="bf16x3",  # noqa
                                         b_planes=pl)
            fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.reps):
                fn()
            e1.record()
            torch.cuda.synchronize()
            times[p].append(e0.elapsed_time(e1) / a.reps)
    for p in a.libs:
        ms = statistics.median(times[p])
        print(f"{p:28s} {a.case} median {ms:6.3f} ms  ({6 * 2.0 * D * D * T / ms / 1e9:6.1f} hwTF)  runs "
              f"{' '.join('%.3f' % x for x in times[p])}", flush=True)


if __name__ == "__main__":
    main()
