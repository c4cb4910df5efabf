"""A/B of the tail segmented reduction (tail_seg_reduce_kernel: dP_r[t] = sum_e W[e,r] do[e], dWedge[e,r] =
do[e].P_r[t], dsum[t] = sum_e do[e]) across library builds, at the config-3 shape (R = 2, fp32 rows, T = 4M,
N = 100k) and a config-5 shape (R = 8, bf16 rows, per-edge W, degree 50; T = 20M, N = 400k).  Each build's
outputs are compared bitwise with the first build's.

usage: python tools/bench_tailseg.py lib1.so [lib2.so ...]
"""
import sys

import torch

sys.path.insert(0, ".")
from iddgcn_amd import _lib as L  # noqa: E402
from iddgcn_amd import ops  # noqa: E402
from tools.bench_mem import load_lenient, timeit  # noqa: E402


def case(T, N, R, D, bf16, dsum, seed=0):
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(seed)
    t = torch.sort(torch.randint(0, N, (T,), device=dev, generator=g)).values
    cnt = torch.bincount(t, minlength=N)
    x = {"tptr": torch.cat([torch.zeros(1, dtype=torch.long, device=dev), torch.cumsum(cnt, 0)]).int(),
         "W": torch.rand(T, R, device=dev, generator=g),
         "dO": torch.randn(T, D, device=dev, generator=g) * 1e-3,
         "P": torch.randn(R, N, D, device=dev, generator=g),
         "dP": torch.empty(R, N, D, device=dev), "dW": torch.empty(T, R, device=dev),
         "dsum": torch.empty(N, D, device=dev) if dsum else None}
    if bf16:
        x["dO"] = x["dO"].to(torch.bfloat16)
    x["bytes"] = T * D * (2 if bf16 else 4) + T * R * 8 + R * N * D * 8 + (N * D * 4 if dsum else 0)
    return x


def run(x):
    ops.tail_seg_reduce(x["tptr"], None, x["W"], x["dO"], x["P"], x["dP"], x["dW"], dsum=x["dsum"])


def dm_case(T, N, R, D, bf16, seed=0):
    """DistMult + BCE + both seeds by head segment (distmult_heads_kernel)."""
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(seed)
    h = torch.randint(0, N, (T,), device=dev, generator=g)
    hperm = torch.argsort(h, stable=True)
    x = {"hptr": torch.searchsorted(h[hperm], torch.arange(N + 1, device=dev), right=False).int(),
         "hperm": hperm.int(), "Xh": torch.rand(N, D, device=dev, generator=g),
         "Xt": torch.rand(T, D, device=dev, generator=g), "r": torch.randint(0, R, (T,), device=dev, generator=g).int(),
         "rel": torch.rand(R, D, device=dev, generator=g), "y": (torch.rand(T, device=dev, generator=g) > 0.5).float(),
         "dXh": torch.empty(N, D, device=dev)}
    if bf16:
        x["Xt"] = x["Xt"].to(torch.bfloat16)
    x["do"] = torch.empty_like(x["Xt"])
    nb = ops.distmult_blocks(T)
    x["drel"], x["loss"] = torch.empty(nb * R * D, device=dev), torch.empty(nb, device=dev)
    x["bytes"] = 2 * T * D * (2 if bf16 else 4) + 2 * N * D * 4
    return x


def dm_run(x):
    ops.distmult_bce_heads(x["hptr"], x["hperm"], x["Xh"], x["Xt"], x["r"], x["rel"], x["y"], x["do"], x["dXh"],
                           x["drel"], x["loss"], scale=1e-5)


def sweep(name, x, fn, outs):
    ref = None
    for p in sys.argv[1:]:
        L._lib = load_lenient(p)
        ms = timeit(lambda: fn(x))
        out = [o.clone() for o in outs(x)]
        same = "ref" if ref is None else ("bitwise" if all(torch.equal(a, b) for a, b in zip(out, ref)) else "DIFFERS")
        ref = ref or out
        print(f"{name:18s} {p.split('/')[-1]:14s} {ms:7.3f} ms  {x['bytes'] / ms / 1e9:5.2f} TB/s  {same}", flush=True)


if __name__ == "__main__":
    for name, shp in {"dm_cfg3_R2_f32": (4_000_000, 100_000, 2, 256, False),
                      "dm_cfg5_R8_bf16": (20_000_000, 400_000, 8, 256, True)}.items():
        x = dm_case(*shp)
        sweep(name, x, dm_run, lambda x: [x["do"], x["dXh"], x["drel"], x["loss"]])
        del x
        torch.cuda.empty_cache()
    shapes = {"cfg3_R2_f32": (4_000_000, 100_000, 2, 256, False, False),
              "cfg3_R2_f32_dsum": (4_000_000, 100_000, 2, 256, False, True),
              "cfg5_R8_bf16": (20_000_000, 400_000, 8, 256, True, False)}
    for name, shp in shapes.items():
        x = case(*shp)
        ref = None
        for p in sys.argv[1:]:
            L._lib = load_lenient(p)
            ms = timeit(lambda: run(x))
            out = [x["dP"].clone(), x["dW"].clone()] + ([x["dsum"].clone()] if x["dsum"] is not None else [])
            same = "ref" if ref is None else ("bitwise" if all(torch.equal(a, b) for a, b in zip(out, ref)) else "DIFFERS")
            ref = ref or out
            print(f"{name:18s} {p.split('/')[-1]:14s} {ms:7.3f} ms  {x['bytes'] / ms / 1e9:5.2f} TB/s  {same}", flush=True)
        del x
        torch.cuda.empty_cache()
