"""Per-phase timing of sigma_tn_b3_kernel's loop from the s_memtime stamps of
`tools/runs/dbg/stamp_patch.py OUT sigma_tn` (config-3 shape: M = 4M fp32 rows, D = 256).

Prints, for waves 0 and 4 (one SIMD) of workgroups 0..15, the median cycles of each phase over tiles 2..14, the
offsets of both waves' phase ends from wave 0's loop top, and the core clock (s_memtime ticks per 10 ns
s_memrealtime tick, tile to tile).  X is restored before every launch so the data stay random.

usage: python tools/runs/dbg/stamp_sigma_tn.py STAMP_LIB
"""
import ctypes
import statistics
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from iddgcn_amd import _lib as L  # noqa: E402
from iddgcn_amd import ops  # noqa: E402
from tools.bench_mem import load_lenient  # noqa: E402

PH = ["stage", "sigma' MFMA", "epilogue", "TN MFMA (issue)", "convert + waits", "barrier"]


def main():
    dev = torch.device("cuda", 0)
    M, D = 4_000_000, 256
    g = torch.Generator(device=dev).manual_seed(0)
    X0 = torch.rand(M, D, device=dev, generator=g)
    dO = torch.randn(M, D, device=dev, generator=g) * 1e-3
    S = torch.randn(D, D, device=dev, generator=g) / 16
    X = X0.clone()
    dS = torch.empty(D, D, device=dev)
    slab = torch.empty(ops.sigma_tn_slab_floats(M), device=dev)
    res = {}
    for name, lib in (("product", L.load()), ("stamped", load_lenient(sys.argv[1]))):
        L._lib = lib
        ts = []
        for _ in range(6):
            X.copy_(X0)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            ops.sigma_tn(dO, X, S, dS, slab, precision="bf16x3")
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        res[name] = (statistics.median(ts[1:]), X.clone(), dS.clone())
    same = torch.equal(res["product"][1], res["stamped"][1]) and torch.equal(res["product"][2], res["stamped"][2])
    print(f"sigma_tn_b3: product {res['product'][0]:.3f} ms, stamped {res['stamped'][0]:.3f} ms, bitwise equal: {same}")
    lib = L._lib
    buf = np.zeros(32 * 16 * 8, dtype=np.uint64)
    assert lib.iddgcn_dbg_stamps(ctypes.c_void_p(buf.ctypes.data), ctypes.c_longlong(buf.nbytes)) == 0
    s = buf.reshape(32, 16, 8).astype(np.int64)
    for w, label in ((0, "wave 0"), (1, "wave 4")):
        rows = {n: [] for n in PH}
        tot, clk = [], []
        for wg in range(16):
            for t in range(2, 14):
                v = s[wg * 2 + w, t]
                if not v[0] or not v[6]:
                    continue
                for k, n in enumerate(PH):
                    rows[n].append(v[k + 1] - v[k])
                nxt = s[wg * 2 + w, t + 1]
                if nxt[0] and nxt[7] > v[7]:
                    tot.append(nxt[0] - v[0])
                    clk.append((nxt[0] - v[0]) / (nxt[7] - v[7]) * 0.1)
        print(f"  {label}: " + ", ".join(f"{n} {statistics.median(r):.0f}" for n, r in rows.items() if r) +
              (f" | tile {statistics.median(tot):.0f} cycles, clock {statistics.median(clk):.2f} GHz" if tot else ""))
    offs = []
    for wg in range(16):
        for t in range(2, 14):
            a, b = s[wg * 2, t], s[wg * 2 + 1, t]
            if a[0] and b[0]:
                offs.append([a[k] - a[0] for k in range(1, 7)] + [b[k] - a[0] for k in range(0, 7)])
    if offs:
        med = [statistics.median(o[i] for o in offs) for i in range(13)]
        print("  wave 0 phase ends from its top: " + ", ".join(f"{n} {m:.0f}" for n, m in zip(PH, med[:6])))
        print("  wave 4 top {:.0f}; phase ends: ".format(med[6]) + ", ".join(f"{n} {m:.0f}" for n, m in zip(PH, med[7:])))


if __name__ == "__main__":
    main()
