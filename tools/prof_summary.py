"""Summarise a rocprofv3 --kernel-trace --stats CSV: per-kernel calls, total and average time."""
import sys

import pandas as pd


def main(path, steps=None):
    s = pd.read_csv(path)
    s["Kernel"] = s["Name"].str.replace(r"\(anonymous namespace\)::", "", regex=True).str.slice(0, 60)
    s["TotalMs"] = s["TotalDurationNs"] / 1e6
    s["AvgUs"] = s["AverageNs"] / 1e3
    cols = ["Kernel", "Calls", "TotalMs", "AvgUs", "Percentage"]
    if steps:
        s["MsPerStep"] = s["TotalMs"] / steps
        cols.append("MsPerStep")
    print(s[cols].to_string(index=False, float_format=lambda x: f"{x:.3f}"))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else None)
