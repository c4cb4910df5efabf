"""Time the edge-level memory-bound kernels alone at config-3 shape (T = 4M edges, D = 256, R = 2),
beside torch fill / copy of the same byte counts (what the box's HBM sustains for that pattern).

usage: python tools/bench_mem.py [libpath ...]   (each lib is loaded in turn, same inputs)
"""
import sys

import torch

sys.path.insert(0, ".")
from iddgcn_amd import _lib as L  # noqa: E402
from iddgcn_amd import ops  # noqa: E402


def timeit(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def inputs(T=4_000_000, N=100_000, D=256, R=2):
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    x = {}
    x["A"] = torch.rand(T, D, device=dev, generator=g)
    x["B"] = torch.rand(T, D, device=dev, generator=g)
    x["C"] = torch.empty(T, D, device=dev)
    x["Wedge"] = torch.rand(T, R, device=dev, generator=g)
    x["P"] = torch.randn(R, N, D, device=dev, generator=g)
    x["Y"] = torch.randn(N, D, device=dev, generator=g)
    x["Xh"] = torch.rand(N, D, device=dev, generator=g)
    x["rel"] = torch.rand(R, D, device=dev, generator=g)
    t = torch.sort(torch.randint(0, N, (T,), device=dev, generator=g)).values
    x["t"] = t.int()
    x["h"] = torch.randint(0, N, (T,), device=dev, generator=g).int()
    x["r"] = torch.randint(0, R, (T,), device=dev, generator=g).int()
    x["y"] = (torch.rand(T, device=dev, generator=g) > 0.5).float()
    cnt = torch.bincount(t, minlength=N)
    x["tptr"] = torch.cat([torch.zeros(1, dtype=torch.long, device=dev), torch.cumsum(cnt, 0)]).int()
    hperm = torch.argsort(x["h"].long(), stable=True)
    x["hperm"] = hperm.int()
    x["hptr"] = torch.searchsorted(x["h"].long()[hperm], torch.arange(N + 1, device=dev), right=False).int()
    x["dXh"] = torch.empty(N, D, device=dev)
    x["dP"] = torch.empty(R, N, D, device=dev)
    x["dW"] = torch.empty(T, R, device=dev)
    x["ds"] = torch.empty(T, device=dev)
    nb = ops.distmult_blocks(T)
    x["drel_slab"] = torch.empty(nb * R * D, device=dev)
    x["loss_slab"] = torch.empty(nb, device=dev)
    x["T"], x["N"], x["D"], x["R"] = T, N, D, R
    return x


def load_lenient(path):
    """Bind the symbols a variant build has (older sources may lack newer entry points)."""
    import ctypes
    lib = ctypes.CDLL(path)
    for name, (res, args) in L.SIGNATURES.items():
        if hasattr(lib, name):
            fn = getattr(lib, name)
            fn.restype, fn.argtypes = res, args
    return lib


def run(libpath, x):
    L._lib = load_lenient(libpath)
    T, N, D = x["T"], x["N"], x["D"]
    gb = T * D * 4 / 1e9
    cases = {
        # name: (fn, HBM GB of the streamed rows)
        "fill": (lambda: x["C"].fill_(1.0), gb),
        "copy": (lambda: x["C"].copy_(x["A"]), 2 * gb),
        "combine": (lambda: ops.combine(x["Y"], x["Wedge"], x["P"], x["C"], y_idx=x["t"], v_idx=x["t"]), gb),
        "combine_R0": (lambda: ops.combine(x["Y"], x["Wedge"][:, :0], x["P"][:0], x["C"], y_idx=x["t"]), gb),
        "combine_R2_noidx_Y": (lambda: ops.combine(x["A"], x["Wedge"], x["P"], x["C"], v_idx=x["t"]), 2 * gb),
        "distmult": (lambda: ops.distmult_bce(x["Xh"], x["h"], x["A"], x["r"], x["rel"], y=x["y"], scale=1e-5,
                                              ds_out=x["ds"], do_out=x["C"], drel_slab=x["drel_slab"],
                                              loss_slab=x["loss_slab"]), 2 * gb),
        "dm+seg_gather": (lambda: (ops.distmult_bce(x["Xh"], x["h"], x["A"], x["r"], x["rel"], y=x["y"], scale=1e-5,
                                                    ds_out=x["ds"], do_out=x["C"], drel_slab=x["drel_slab"],
                                                    loss_slab=x["loss_slab"]),
                                   ops.seg_gather_reduce(x["hptr"], x["A"], x["dXh"], perm=x["hperm"], coef=x["ds"],
                                                         r_idx=x["r"], rel=x["rel"], X=x["Xh"])), 3 * gb),
        "dm_heads": (lambda: ops.distmult_bce_heads(x["hptr"], x["hperm"], x["Xh"], x["A"], x["r"], x["rel"], x["y"],
                                                    x["C"], x["dXh"], x["drel_slab"], x["loss_slab"], scale=1e-5),
                     2 * gb),
        "tail_seg": (lambda: ops.tail_seg_reduce(x["tptr"], None, x["Wedge"], x["A"], x["P"], x["dP"], x["dW"]), gb),
    }
    res = []
    for name, (fn, b) in cases.items():
        ms = timeit(fn)
        res.append(f"{name}={ms:.3f}ms/{b / ms:.2f}TB/s")
    print(libpath.split("/")[-1], " ".join(res), flush=True)


if __name__ == "__main__":
    x = inputs()
    for p in sys.argv[1:] or [L.LIB_PATH]:
        run(p, x)
