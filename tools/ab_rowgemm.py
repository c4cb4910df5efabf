"""A/B timing of the D=256 row-GEMM forms of a training step across builds of libiddgcn_hip.so.

Every library is driven through its own iddgcn_rowgemm_f32 entry point (the iddgcn_rowgemm_t layout
is unchanged since ABI 2, so older builds load too), on the same inputs, in split-fp16 mode, at the
config-3 shapes: T = 4M edge rows, N = 100k node rows.
usage: python tools/ab_rowgemm.py [--cases fwd,bwd,...] [--rounds K] lib_a.so [lib_b.so ...]
(the libraries are timed round-robin, K rounds, 10 launches each; the per-case median over rounds is printed)
"""
import ctypes
import sys

import torch

sys.path.insert(0, ".")
from iddgcn_amd import _lib as L  # noqa: E402
from iddgcn_amd import ops  # noqa: E402


def load(path):
    lib = ctypes.CDLL(path)
    lib.iddgcn_rowgemm_f32.argtypes = [ctypes.c_void_p, ctypes.POINTER(L.RowGemmArgs)]
    lib.iddgcn_rowgemm_f32.restype = ctypes.c_int
    lib.iddgcn_set_gemm_precision.argtypes = [ctypes.c_int]
    return lib


def main(paths, reps=10, rounds=3, only=None):
    dev = torch.device("cuda", 0)
    T, N, D, R = 4_000_000, 100_000, 256, 2
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.rand(T, D, device=dev, generator=g)
    do = torch.randn(T, D, device=dev, generator=g) * 1e-6
    C = torch.empty(T, D, device=dev)
    S = torch.randn(D, D, device=dev, generator=g) / 16
    W = torch.rand(T, R, device=dev, generator=g)
    P = torch.randn(R, N, D, device=dev, generator=g)
    t = torch.sort(torch.randint(0, N, (T,), device=dev, generator=g)).values.int()
    Xn = torch.rand(N, D, device=dev, generator=g)
    dOn = torch.randn(N, D, device=dev, generator=g)
    Cn = torch.empty(N, D, device=dev)
    dz = torch.randn(N, R, device=dev, generator=g)
    WaT = torch.randn(R, D, device=dev, generator=g)
    xin = x.clone()
    xpl = ops.f32_to_planes(x)                # pre-split planes tables (IDDGCN_PLANES_*)
    xpl_in = xpl.clone()
    Cpl = torch.empty_like(xpl)
    cases = {
        "fwd": ("fwd_combine (T)", x, S, C, dict(coef=W, V=P, v_idx=t, v_rel_stride=N * D, act=L.ACT_SIGMOID)),
        "bwd": ("bwd_dsig separate C (T)", do, S, C, dict(b_trans=True, act=L.ACT_DSIGMOID, aux=x)),
        "bwdip": ("bwd_dsig C = aux (T)", do, S, xin, dict(b_trans=True, act=L.ACT_DSIGMOID, aux=xin)),
        "bwdpl": ("bwd_dsig planes aux, C = aux (T)", do, S, xpl_in,
                  dict(b_trans=True, act=L.ACT_DSIGMOID, aux=xpl_in, planes=L.PLANES_AUX)),
        "fwdpl": ("fwd_combine planes A+C (T)", xpl, S, Cpl, dict(coef=W, V=P, v_idx=t, v_rel_stride=N * D,
                                                                  act=L.ACT_SIGMOID, planes=L.PLANES_A | L.PLANES_C)),
        "fwdpa": ("fwd_combine planes A (T)", xpl, S, C, dict(coef=W, V=P, v_idx=t, v_rel_stride=N * D,
                                                              act=L.ACT_SIGMOID, planes=L.PLANES_A)),
        "nbd": ("node bcast+dsig (N)", dOn, S, Cn, dict(b_trans=True, coef=dz, V=WaT, v_rel_stride=D, v_row_stride=0,
                                                        act=L.ACT_DSIGMOID, aux=Xn)),
        "nb": ("node bcast (N)", dOn, S, Cn, dict(b_trans=True, coef=dz, V=WaT, v_rel_stride=D, v_row_stride=0)),
        "np": ("node plain (N)", Xn, S, Cn, dict()),
    }
    if only:
        cases = {k: v for k, v in cases.items() if k in only}
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    libs = [load(p) for p in paths]
    res = {(p, k): [] for p in paths for k in cases}
    for _ in range(rounds):
        for path, lib in zip(paths, libs):
            lib.iddgcn_set_gemm_precision(L.GEMM_SPLIT_F16)
            for k, (name, A, B, Cc, kw) in cases.items():
                args = ops._rowgemm_args(A, B, Cc, **kw)
                for _ in range(2):
                    assert lib.iddgcn_rowgemm_f32(st, ctypes.byref(args)) == 0
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(reps):
                    lib.iddgcn_rowgemm_f32(st, ctypes.byref(args))
                e1.record()
                torch.cuda.synchronize()
                res[(path, k)].append(e0.elapsed_time(e1) / reps * 1e3)
    for path in paths:
        print(f"--- {path}", flush=True)
        for k, (name, *_r) in cases.items():
            v = sorted(res[(path, k)])
            print(f"{name:28s} {v[len(v) // 2]:9.1f} us   (min {v[0]:.1f}, max {v[-1]:.1f})", flush=True)


if __name__ == "__main__":
    argv = sys.argv[1:]
    only, rounds = None, 3
    while argv and argv[0].startswith("--"):
        if argv[0] == "--cases":
            only = argv[1].split(",")
        elif argv[0] == "--rounds":
            rounds = int(argv[1])
        argv = argv[2:]
    main(argv, rounds=rounds, only=only)
