"""Per-kernel-class PMC summary from rocprofv3 --pmc CSVs (last training step of a bench run).

Reports: duration, effective clock (GRBM_GUI_ACTIVE / 8 XCDs / duration, MI355X_MICROARCH.md DVFS
note), MFMA busy fraction, and HBM bytes (FETCH_SIZE x2 on gfx950 for wide streaming reads +
WRITE_SIZE, KiB units) per dispatch.
"""
import sys

import pandas as pd


def load(path):
    c = pd.read_csv(path)
    c["dur_us"] = (c["End_Timestamp"] - c["Start_Timestamp"]) / 1e3
    w = c.pivot_table(index=["Dispatch_Id", "Kernel_Name", "Grid_Size", "dur_us"], columns="Counter_Name",
                      values="Counter_Value", aggfunc="sum").reset_index()
    w["kernel"] = w["Kernel_Name"].str.replace(r"\(anonymous namespace\)::", "", regex=True).str.slice(0, 48)
    return w.sort_values("Dispatch_Id")


def main(d1, d2=None, d3=None):
    w = load(f"{d1}/run_counter_collection.csv")
    if d2:
        f = load(f"{d2}/run_counter_collection.csv")[["Dispatch_Id", "FETCH_SIZE"]]
        w = w.merge(f, on="Dispatch_Id", how="left")
    if d3:
        f = load(f"{d3}/run_counter_collection.csv")[["Dispatch_Id", "WRITE_SIZE"]]
        w = w.merge(f, on="Dispatch_Id", how="left")
    ad = w.index[w["kernel"].str.contains("adam")].tolist()
    step = w.loc[ad[-3] + 1: ad[-1]] if len(ad) >= 3 else w
    step = step.copy()
    step["clk_GHz"] = step["GRBM_GUI_ACTIVE"] / 8 / (step["dur_us"] * 1e3)
    if "SQ_VALU_MFMA_BUSY_CYCLES" in step:
        # MFMA busy cycles summed over all SIMDs (1024) vs elapsed shader cycles
        step["mfma_busy"] = step["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * step["GRBM_GUI_ACTIVE"] / 8)
    if "FETCH_SIZE" in step:
        step["read_GB"] = step["FETCH_SIZE"] * 2 * 1024 / 1e9
    if "WRITE_SIZE" in step:
        step["write_GB"] = step["WRITE_SIZE"] * 1024 / 1e9
    cols = [c for c in ["kernel", "Grid_Size", "dur_us", "clk_GHz", "mfma_busy", "read_GB", "write_GB"] if c in step]
    print(step[cols].to_string(index=False, float_format=lambda x: f"{x:.3f}"))


if __name__ == "__main__":
    main(*sys.argv[1:])
