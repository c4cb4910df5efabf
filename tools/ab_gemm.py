"""A/B of the D = 256 edge GEMM kernels across library builds, on identical inputs (config-3 shape by default).

For every library (built variants of the same C-ABI) and every case (the bf16x3 forms the engine launches at
config 3, plus the exact forms for reference), it times `reps` launches (HIP events, after one warm launch), and
compares each case's output with the FIRST library's output bitwise (max |diff| reported when not equal) and with a
float64 reference on the first `check` rows.  The libraries alternate `rounds` times so a drifting clock hits every
build alike; the per-library median is reported.

usage: python tools/ab_gemm.py [--T 4000000] [--modes bf16x3] [--cases fwd_combine,bwd_dsig,plain,acc,bc,tn]
                              [--rounds 3] lib1.so lib2.so ...
"""
import argparse
import statistics
import sys

import torch

sys.path.insert(0, ".")
from iddgcn_amd import _lib as L  # noqa: E402
from iddgcn_amd import ops  # noqa: E402


def make_inputs(T, N, D, R, dev):
    g = torch.Generator(device=dev).manual_seed(0)
    x = {}
    x["A"] = torch.rand(T, D, device=dev, generator=g)
    x["S"] = torch.randn(D, D, device=dev, generator=g)
    W = torch.rand(N, R, device=dev, generator=g)
    h = torch.randint(0, N, (T,), device=dev, generator=g)
    x["Wedge"] = W[h].contiguous()
    x["P"] = torch.randn(R, N, D, device=dev, generator=g) * 4
    x["t"] = torch.sort(torch.randint(0, N, (T,), device=dev, generator=g)).values.int()
    x["aux"] = torch.rand(T, D, device=dev, generator=g)
    x["dO"] = torch.randn(T, D, device=dev, generator=g) * 1e-3
    x["C"] = torch.empty(T, D, device=dev)
    x["C0"] = torch.randn(T, D, device=dev, generator=g)
    x["slab"] = torch.empty(ops.tn_blocks(T, D) * D * D, device=dev)
    x["dS"] = torch.empty(D, D, device=dev)
    x["dz"] = torch.randn(T, R, device=dev, generator=g)
    x["WaT"] = torch.randn(R, D, device=dev, generator=g)
    return x


def cases(x, N, D, mode):
    A, S, C = x["A"], x["S"], x["C"]
    return {
        "fwd_combine": (lambda: ops.rowgemm(A, S, C, coef=x["Wedge"], V=x["P"], v_idx=x["t"], v_rel_stride=N * D,
                                            act=L.ACT_SIGMOID, precision=mode), C),
        "bwd_dsig": (lambda: ops.rowgemm(x["dO"], S, C, b_trans=True, act=L.ACT_DSIGMOID, aux=x["aux"],
                                         precision=mode), C),
        "plain": (lambda: ops.rowgemm(A, S, C, precision=mode), C),
        "acc": (lambda: (C.copy_(x["C0"]), ops.rowgemm(A, S, C, accumulate=True, b_trans=True, precision=mode)), C),
        "bc": (lambda: ops.rowgemm(x["dO"], S, C, b_trans=True, coef=x["dz"], V=x["WaT"], v_rel_stride=D,
                                   v_row_stride=0, act=L.ACT_DSIGMOID, aux=x["aux"], precision=mode), C),
        "tn": (lambda: ops.gemm_tn(A, x["dO"], x["dS"], x["slab"], precision=mode), x["dS"]),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", type=int, default=4_000_000)
    ap.add_argument("--N", type=int, default=100_000)
    ap.add_argument("--modes", default="bf16x3")
    ap.add_argument("--cases", default="fwd_combine,bwd_dsig,plain,acc,bc,tn")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("libs", nargs="+")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    D, R = 256, 2
    x = make_inputs(a.T, a.N, D, R, dev)
    libs = [L.load(p) for p in a.libs]
    want = a.cases.split(",")
    times, outs = {}, {}
    for rnd in range(a.rounds):
        for li, lib in enumerate(libs):
            L._lib = lib
            for mode in a.modes.split(","):
                for name, (fn, out) in cases(x, a.N, D, mode).items():
                    if name not in want:
                        continue
                    fn()
                    torch.cuda.synchronize()
                    if rnd == 0:
                        outs[(li, mode, name)] = out.detach().clone()
                    if name == "acc":       # timing the C += A B form re-accumulates: restore C first each launch
                        ev = []
                        for _ in range(a.reps):
                            C0 = x["C0"]
                            x["C"].copy_(C0)
                            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                            e0.record()
                            ops.rowgemm(x["A"], x["S"], x["C"], accumulate=True, b_trans=True, precision=mode)
                            e1.record()
                            ev.append((e0, e1))
                        torch.cuda.synchronize()
                        ms = statistics.mean(e0.elapsed_time(e1) for e0, e1 in ev)
                    else:
                        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                        e0.record()
                        for _ in range(a.reps):
                            fn()
                        e1.record()
                        torch.cuda.synchronize()
                        ms = e0.elapsed_time(e1) / a.reps
                    times.setdefault((li, mode, name), []).append(ms)
    hw = {"bf16x3": 6, "split": 3, "exact": 1}
    for (li, mode, name), ts in sorted(times.items(), key=lambda kv: (kv[0][1], kv[0][2], kv[0][0])):
        med = statistics.median(ts)
        ref = outs[(0, mode, name)]
        o = outs[(li, mode, name)]
        same = torch.equal(o, ref)
        diff = "bitwise" if same else f"maxdiff={((o - ref).abs().max() / ref.abs().max()).item():.2e}"
        flop = 2.0 * D * D * a.T * hw[mode]
        print(f"{a.libs[li]:28s} {mode:6s} {name:12s} median {med:7.3f} ms  (runs {' '.join(f'{t:.3f}' for t in ts)})"
              f"  {flop / med / 1e9:7.1f} hwTF  vs lib0: {diff}", flush=True)


if __name__ == "__main__":
    main()
