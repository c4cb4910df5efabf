"""Cross-check bench.py's roofline line against a rocprofv3 kernel trace of the same command.

bench.py times the dominant kernel's EDGE-level launches with HIP events; the same kernel symbol
also runs small node-level launches, so rocprof's per-symbol average mixes both.  This script
reads run_kernel_trace.csv, keeps launches of the named kernel whose duration is at least
`frac` of the longest one (the edge-level launches), drops the warm-up steps, and prints
their average next to the bench JSON's avg_launch_ms.

usage: python tools/prof_roofline.py TRACE_CSV BENCH_JSON [kernel_substring]
"""
import json
import sys

import pandas as pd


def main(trace, bench, name="rowgemm256_v3_kernel<2, false, true, false, false, false, false, false>", frac=0.5):
    t = pd.read_csv(trace)
    k = t[t["Kernel_Name"].str.contains(name, regex=False)].copy()
    k["ms"] = (k["End_Timestamp"] - k["Start_Timestamp"]) / 1e6
    big = k[k["ms"] >= frac * k["ms"].max()]
    with open(bench) as f:
        line = [ln for ln in f if ln.startswith("{")][-1]
    b = json.loads(line)
    steps, warm = b["steps"], b["warmup"]
    per_step = len(big) // (steps + warm)
    timed = big.iloc[warm * per_step:]
    rl = b["roofline"]
    avg = timed["ms"].mean()
    print(f"kernel            : {name}")
    print(f"edge launches     : {len(big)} ({per_step}/step), timed {len(timed)}")
    print(f"rocprof avg (ms)  : {avg:.4f}  min {timed['ms'].min():.4f}  max {timed['ms'].max():.4f}")
    print(f"bench avg (ms)    : {rl['avg_launch_ms']:.4f}  (HIP events, bench.py --no-cpu-baseline run)")
    if rl.get("unit") == "GB/s":
        print(f"rocprof GB/s      : {rl['bytes_per_launch'] / avg / 1e6:.1f}  vs bench {rl['achieved']:.1f} "
              f"(algorithmic {rl['bytes_per_launch'] / 1e9:.3f} GB per launch)")
    else:
        # achieved is priced on the MFMA work the operand mode issues (bf16x3: 6 products per
        # algorithmic multiply-add); older bench lines carry only the algorithmic count.
        hw = rl.get("hw_flops_per_launch") or rl["achieved"] * 1e9 * rl["avg_launch_ms"]
        print(f"rocprof TFLOP/s   : {hw / avg / 1e9:.1f}  vs bench {rl['achieved']:.1f} "
              f"(hw {hw / 1e12:.3f} TFLOP, algorithmic {rl['flops_per_launch'] / 1e12:.3f} TFLOP per launch)")


if __name__ == "__main__":
    main(*sys.argv[1:4])
