"""Run-to-run determinism of the tail reduction and DistMult at the config-5 / config-3 shapes: each library
runs the same inputs 3 times; every output must be bitwise equal across the runs (and, where the summation
order is unchanged, to the first library's).

usage: python tools/tailseg_det.py lib1.so [lib2.so ...]
"""
import sys

import torch

sys.path.insert(0, ".")
from iddgcn_amd import _lib as L  # noqa: E402
from tools.bench_mem import load_lenient  # noqa: E402
from tools.bench_tailseg import case, dm_case, dm_run, run  # noqa: E402


def check(name, x, fn, outs, libs, burst=1):
    """burst > 1: that many launches back to back (no fill, no synchronisation between them) per run."""
    first = None
    for p in libs:
        L._lib = load_lenient(p)
        res = []
        for _ in range(3):
            for o in outs(x):
                o.fill_(float("nan"))
            for _ in range(burst):
                fn(x)
            torch.cuda.synchronize()
            res.append([o.clone() for o in outs(x)])
        rr = [all(torch.equal(a, b) for a, b in zip(res[0], r)) for r in res[1:]]
        diffs = []
        for r in res[1:]:
            for k, (a, b) in enumerate(zip(res[0], r)):
                if not torch.equal(a, b):
                    d = (a - b).abs()
                    d = d[torch.isfinite(d)]
                    diffs.append(f"out{k}: {int((a != b).sum())} elems, max {float(d.max()) if d.numel() else float('nan'):.3e}")
        vs_first = "" if first is None else (" same as first lib" if all(torch.equal(a, b) for a, b in zip(first, res[0]))
                                             else " differs from first lib")
        first = first or res[0]
        print(f"{name:18s} {p.split('/')[-1]:14s} run-to-run {'bitwise' if all(rr) else 'DIFFERS ' + '; '.join(diffs)}{vs_first}",
              flush=True)


if __name__ == "__main__":
    libs = sys.argv[1:]
    x = case(20_000_000, 400_000, 8, 256, True, False)
    check("cfg5_R8_bf16 x6", x, run, lambda x: [x["dP"], x["dW"]], libs, burst=6)
    del x
    torch.cuda.empty_cache()
    for name, shp in {"cfg5_R8_bf16": (20_000_000, 400_000, 8, 256, True, False),
                      "cfg5_R8_f32": (4_000_000, 100_000, 8, 256, False, False),
                      "R4_f32": (4_000_000, 100_000, 4, 256, False, False),
                      "cfg3_R2_f32_dsum": (4_000_000, 100_000, 2, 256, False, True)}.items():
        x = case(*shp)
        check(name, x, run, lambda x: [x["dP"], x["dW"]] + ([x["dsum"]] if x["dsum"] is not None else []), libs)
        del x
        torch.cuda.empty_cache()
    for name, shp in {"dm_cfg3_R2_f32": (4_000_000, 100_000, 2, 256, False),
                      "dm_cfg5_R8_bf16": (20_000_000, 400_000, 8, 256, True)}.items():
        x = dm_case(*shp)
        check(name, x, dm_run, lambda x: [x["do"], x["dXh"], x["drel"], x["loss"]], libs)
        del x
        torch.cuda.empty_cache()
