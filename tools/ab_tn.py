"""A/B timing of the D=256 dS TN GEMM (x planes ^T . do, split mode) across builds of libiddgcn_hip.so at the
config-3 shape (T = 4M rows).  usage: python tools/ab_tn.py [--rounds K] lib_a.so [lib_b.so ...]"""
import ctypes
import sys

import torch

sys.path.insert(0, ".")
from iddgcn_amd import _lib as L  # noqa: E402
from iddgcn_amd import ops  # noqa: E402


def main(paths, reps=10, rounds=3):
    dev = torch.device("cuda", 0)
    T, D = 4_000_000, 256
    g = torch.Generator(device=dev).manual_seed(0)
    xpl = ops.f32_to_planes(torch.rand(T, D, device=dev, generator=g))
    do = torch.randn(T, D, device=dev, generator=g) * 1e-6
    C = torch.empty(D, D, device=dev)
    nb = ops.tn_blocks(T, D)
    slab = torch.empty(nb * D * D, device=dev)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    libs = []
    for p in paths:
        lib = ctypes.CDLL(p)
        fn = lib.iddgcn_gemm_tn_planes_f32
        fn.restype, fn.argtypes = L.SIGNATURES["iddgcn_gemm_tn_planes_f32"]
        lib.iddgcn_set_gemm_precision.argtypes = [ctypes.c_int]
        libs.append((p, lib, fn))
    res = {p: [] for p in paths}
    args = None
    for _ in range(rounds):
        for p, lib, fn in libs:
            lib.iddgcn_set_gemm_precision(L.GEMM_SPLIT_F16)
            call = lambda: fn(st, T, D, ops._ptr(xpl), ops._ptr(do), ops._ptr(slab), nb, ops._ptr(C), 0)  # noqa: E731
            for _ in range(2):
                call()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                call()
            e1.record()
            torch.cuda.synchronize()
            res[p].append(e0.elapsed_time(e1) / reps * 1e3)
    for p in paths:
        v = sorted(res[p])
        print(f"{p:28s} dS TN planes {v[len(v) // 2]:9.1f} us (min {v[0]:.1f}, max {v[-1]:.1f})", flush=True)


if __name__ == "__main__":
    argv = sys.argv[1:]
    rounds = 3
    if argv and argv[0] == "--rounds":
        rounds, argv = int(argv[1]), argv[2:]
    main(argv, rounds=rounds)
