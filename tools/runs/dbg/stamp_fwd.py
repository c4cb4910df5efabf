"""Per-phase timing of rowgemm256_b3_kernel's main loop from the s_memtime stamps of tools/runs/dbg/stamp_patch.py.

Runs one case of tools/ab_gemm.py (config-3 shape) with the instrumented library, reads the stamp table and prints,
for the early (wave 0) and late (wave 4) wave of SIMD 0 in workgroups 0..15, the median cycles of each phase over
tiles 2..15, the core clock (s_memtime ticks per s_memrealtime tick x 100 MHz), and the launch time of the product
library beside the instrumented one.

usage: python tools/runs/dbg/stamp_fwd.py STAMP_LIB [--case fwd_combine]
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
    ap.add_argument("--T", type=int, default=4_000_000)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    N, D = 100_000, 256
    x = make_inputs(a.T, N, D, 2, dev)
    fn, out = cases(x, N, D, "bf16x3")[a.case]
    L._lib = L.load()
    t_prod = timeit(fn)
    ref = out.clone()
    lib = load_lenient(a.lib)
    L._lib = lib
    t_stamp = timeit(fn)
    same = torch.equal(out, ref)
    buf = np.zeros(32 * 16 * 8, dtype=np.uint64)
    lib.iddgcn_dbg_stamps.restype = ctypes.c_int
    rc = lib.iddgcn_dbg_stamps(ctypes.c_void_p(buf.ctypes.data), ctypes.c_longlong(buf.nbytes))
    assert rc == 0, rc
    s = buf.reshape(32, 16, 8).astype(np.int64)
    print(f"case {a.case}: product {t_prod:.3f} ms, instrumented {t_stamp:.3f} ms, output bitwise equal: {same}")
    names = ["pre (top -> MFMA)", "MFMA phase", "post (MFMA -> barrier)", "barrier wait", "tile total"]
    for w, label in ((0, "early wave 0"), (1, "late wave 4")):
        rows = {n: [] for n in names}
        clk = []
        for wg in range(16):
            for t in range(2, 15):
                v = s[wg * 2 + w, t]
                if v[0] == 0 or v[4] == 0:
                    continue
                rows[names[0]].append(v[1] - v[0])
                rows[names[1]].append(v[2] - v[1])
                rows[names[2]].append(v[3] - v[2])
                rows[names[3]].append(v[4] - v[3])
                rows[names[4]].append(v[4] - v[0])
                if v[6] > v[5]:
                    clk.append((v[4] - v[0]) / (v[6] - v[5]) * 100e6 / 1e9)
        print(f"  {label}: " + ", ".join(f"{n} {statistics.median(r):.0f}" for n, r in rows.items() if r) +
              (f"  | clock {statistics.median(clk):.2f} GHz (n={len(clk)})" if clk else ""))
    # the same SIMD's two waves side by side: MFMA phase start/end offsets from the early wave's loop top
    offs = []
    for wg in range(16):
        for t in range(2, 15):
            e, l = s[wg * 2, t], s[wg * 2 + 1, t]
            if e[0] and l[0]:
                offs.append((l[0] - e[0], e[1] - e[0], e[2] - e[0], l[1] - e[0], l[2] - e[0], e[3] - e[0], l[3] - e[0],
                             e[4] - e[0]))
    if offs:
        med = [statistics.median(o[i] for o in offs) for i in range(8)]
        print("  offsets from early top (median cycles): late top {:.0f}, early MFMA {:.0f}-{:.0f}, late MFMA {:.0f}-{:.0f}, "
              "early post done {:.0f}, late post done {:.0f}, barrier exit {:.0f}".format(*med))


if __name__ == "__main__":
    main()
