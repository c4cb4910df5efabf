"""Fine phase stamps of rowgemm256_b3_kernel's loop (`tools/runs/dbg/stamp_patch.py OUT rowgemm_fine`): for the early
(wave 0) and late (wave 4) wave of SIMD 0, workgroups 0..15, tiles 2..14, the median offset of each stamp from the
early wave's loop top (cycles).  Stamps: 0 top, 1 after the A DMAs, late: 2 slabs waited, 3 epilogue(t-1), 4 slab
DMAs(t), 5 idx DMA(t+1); 6 MFMA start, 7 MFMA end; late: 8 A waited, 9 converted; early: 8 slabs waited,
9 epilogue(t), 10 A waited, 11 converted, 12 slab DMAs(t+1), 13 idx DMA(t+2); 14 before the barrier, 15 after it.

usage: python tools/runs/dbg/stamp_fwd_fine.py STAMP_LIB [--case fwd_combine]
"""
import argparse
import ctypes
import statistics
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from iddgcn_amd import _lib as L  # noqa: E402
from tools.ab_gemm import cases, make_inputs  # noqa: E402
from tools.bench_mem import load_lenient, timeit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib")
    ap.add_argument("--case", default="fwd_combine")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    N, D = 100_000, 256
    x = make_inputs(4_000_000, N, D, 2, dev)
    fn, out = cases(x, N, D, "bf16x3")[a.case]
    L._lib = L.load()
    t_prod = timeit(fn)
    lib = load_lenient(a.lib)
    L._lib = lib
    t_stamp = timeit(fn)
    buf = np.zeros(32 * 16 * 16, dtype=np.uint64)
    assert lib.iddgcn_dbg_stamps(ctypes.c_void_p(buf.ctypes.data), ctypes.c_longlong(buf.nbytes)) == 0
    s = buf.reshape(32, 16, 16).astype(np.int64)
    print(f"case {a.case}: product {t_prod:.3f} ms, stamped {t_stamp:.3f} ms")
    for w, label in ((0, "early wave 0"), (1, "late wave 4")):
        meds = []
        for k in range(16):
            vals = [s[wg * 2 + w, t, k] - s[wg * 2, t, 0] for wg in range(16) for t in range(2, 15)
                    if s[wg * 2, t, 0] and s[wg * 2 + w, t, k]]
            meds.append(f"{k}:{statistics.median(vals):.0f}" if vals else f"{k}:-")
        print(f"  {label}: " + " ".join(meds))
    if hasattr(lib, "iddgcn_dbg_rt"):      # s_memrealtime (100 MHz) beside stamps 0 and 15: the in-kernel clock
        br = np.zeros(32 * 16 * 2, dtype=np.uint64)
        assert lib.iddgcn_dbg_rt(ctypes.c_void_p(br.ctypes.data), ctypes.c_longlong(br.nbytes)) == 0
        rt = br.reshape(32, 16, 2).astype(np.int64)
        clk = [(s[j, t, 15] - s[j, t, 0]) / (rt[j, t, 1] - rt[j, t, 0]) * 0.1 for j in range(32) for t in range(2, 15)
               if rt[j, t, 1] > rt[j, t, 0] and s[j, t, 15] and s[j, t, 0]]
        if clk:
            print(f"  in-kernel clock {statistics.median(clk):.3f} GHz (n={len(clk)})")
    if hasattr(lib, "iddgcn_dbg_stampx"):
        bx = np.zeros(32 * 16 * 4, dtype=np.uint64)
        assert lib.iddgcn_dbg_stampx(ctypes.c_void_p(bx.ctypes.data), ctypes.c_longlong(bx.nbytes)) == 0
        x = bx.reshape(32, 16, 4).astype(np.int64)
        # the slab wait split: done when only (A, idx, slabs) / (A, idx) are younger
        for w, ks, label in ((1, (0, 1), "late: older-than-slabs done, slabs done"),
                             (0, (2, 3), "early: older-than-slabs done, slabs done")):
            vals = [[x[wg * 2 + w, t, k] - s[wg * 2, t, 0] for wg in range(16) for t in range(2, 15)
                     if s[wg * 2, t, 0] and x[wg * 2 + w, t, k]] for k in ks]
            print(f"  {label}: " + " ".join(f"{statistics.median(v):.0f}" if v else "-" for v in vals))


if __name__ == "__main__":
    main()
