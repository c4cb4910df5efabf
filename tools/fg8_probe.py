"""The config-5 forward edge GEMM alone (R = 8, bf16 edge tables, T = 50M, N = 1M, tail-sorted rows with runs of
~50): A/B timing across library builds on identical inputs, outputs compared bitwise with the first build's, and a
short fixed run for rocprofv3 --pmc passes.

usage: python tools/fg8_probe.py [reps] [linear] [lib.so | v3 ...]   ("v3": the default library with a coefficient table
that is not 16-B aligned, which sends the call to the older rowgemm256_v3_kernel path)
"""
import sys

import torch

sys.path.insert(0, ".")
from iddgcn_amd import _lib as L  # noqa: E402
from iddgcn_amd import ops  # noqa: E402
from tools.bench_mem import load_lenient  # noqa: E402

T, N, D, R = 50_000_000, 1_000_000, 256, 8


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    libs = sys.argv[2:] or [None]
    act = L.ACT_SIGMOID
    if libs[0] == "linear":                     # no activation (timing the epilogue's sigmoid)
        act, libs = L.ACT_NONE, libs[1:] or [None]
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(5)
    lengths = torch.randint(4, 97, (N,), device=dev, generator=g)
    t = torch.repeat_interleave(torch.arange(N, device=dev, dtype=torch.int32), lengths)[:T]
    t = torch.cat([t, torch.full((T - len(t),), N - 1, device=dev, dtype=torch.int32)]) if len(t) < T else t
    A = torch.empty(T, D, device=dev, dtype=torch.bfloat16)
    for i in range(0, T, 1 << 24):
        A[i:i + (1 << 24)] = torch.rand(min(1 << 24, T - i), D, device=dev, generator=g)
    S = torch.randn(D, D, device=dev, generator=g) / 16
    W = torch.rand(T, R, device=dev, generator=g)
    P = torch.randn(R, N, D, device=dev, generator=g)
    C = torch.empty(T, D, device=dev, dtype=torch.bfloat16)
    Wu = None
    ref = None
    for lp in libs:
        coef = W
        if lp == "v3":
            if Wu is None:
                Wu = torch.empty(T * R + 1, device=dev)[1:].view(T, R)
                Wu.copy_(W)
            coef = Wu
        elif lp:
            L._lib = load_lenient(lp)
        tag = lp.split("/")[-1] if lp else "default"
        run = lambda: ops.rowgemm(A, S, C, coef=coef, V=P, v_idx=t, v_rel_stride=N * D, act=act)  # noqa: E731
        run()
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record()
        for _ in range(reps):
            run()
        ev[1].record()
        torch.cuda.synchronize()
        ms = ev[0].elapsed_time(ev[1]) / reps
        if ref is None:
            ref, same = C[::97].clone(), "ref"
        else:
            same = "bitwise" if torch.equal(C[::97], ref) else \
                f"max diff {(C[::97].float() - ref.float()).abs().max().item():.3e}"
        print(f"{tag:16s} fwd R8 bf16 {ms:8.3f} ms  {61.19e9 / ms / 1e6:7.1f} GB/s  {same}", flush=True)


if __name__ == "__main__":
    main()
