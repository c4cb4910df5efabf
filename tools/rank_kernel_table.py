"""Per-kernel time of one rank's step of a node-row partition beside the single-GPU step (name the
kernels that do not shrink by the partition's factor).  Inputs: two rocprofv3 --kernel-trace --stats CSVs of
tools/node_shard_dryrun.py (ranks "none" = the single-GPU step only, and one rank), each over `steps` training
steps (the tool's warm-up step included), so both are per-step averages of the same kernels.

usage: python tools/rank_kernel_table.py FULL_STATS.csv RANK_STATS.csv STEPS WORLD [top]
"""
import sys

import pandas as pd


def per_step(path, steps):
    s = pd.read_csv(path)
    s["Kernel"] = s["Name"].str.replace(r"\(anonymous namespace\)::", "", regex=True).str.slice(0, 58)
    return s.groupby("Kernel")["TotalDurationNs"].sum() / 1e6 / steps


def main(full, rank, steps, world, top=25):
    f, r = per_step(full, steps), per_step(rank, steps)
    t = pd.DataFrame({"single_gpu_ms": f, "rank_ms": r}).fillna(0.0)
    t["ratio"] = t["single_gpu_ms"] / t["rank_ms"].where(t["rank_ms"] > 0)
    t["excess_ms"] = t["rank_ms"] - t["single_gpu_ms"] / world      # what the rank spends beyond a 1/world share
    t = t.sort_values("excess_ms", ascending=False)
    print(f"per step; rank total {t['rank_ms'].sum():.2f} ms, single-GPU total {t['single_gpu_ms'].sum():.2f} ms "
          f"(1/{world}: {t['single_gpu_ms'].sum() / world:.2f} ms); sorted by the rank's excess over a 1/{world} share")
    print(t.head(top).to_string(float_format=lambda x: f"{x:.3f}"))


if __name__ == "__main__":
    a = sys.argv[1:]
    main(a[0], a[1], int(a[2]), int(a[3]), int(a[4]) if len(a) > 4 else 25)
