"""Summarise tools/pmc_gemm.sh output: per case, the long launches' SQ counters as fractions.

usage: python tools/pmc_sq_summary.py gpurun_out/pmcg case...
"""
import glob
import os
import sys

import pandas as pd


def load(d):
    path = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    c = pd.read_csv(path)
    c["dur_ms"] = (c["End_Timestamp"] - c["Start_Timestamp"]) / 1e6
    w = c.pivot_table(index=["Dispatch_Id", "Kernel_Name", "dur_ms"], columns="Counter_Name",
                      values="Counter_Value", aggfunc="sum").reset_index()
    w = w[w["dur_ms"] >= 0.5 * w["dur_ms"].max()]
    return w.drop(columns=["Dispatch_Id", "Kernel_Name"]).mean(numeric_only=True)


def main(root, *cases):
    for c in cases:
        s = pd.concat([load(os.path.join(root, f"{c}_1")), load(os.path.join(root, f"{c}_2"))])
        s = s[~s.index.duplicated()]
        busy = s["SQ_BUSY_CYCLES"]
        wave = s["SQ_WAVE_CYCLES"]
        print(f"== {c}: {s['dur_ms']:.3f} ms; clock {s['GRBM_GUI_ACTIVE'] / 8 / (s['dur_ms'] * 1e6):.2f} GHz")
        for k in ["SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                  "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_VMEM", "SQ_WAIT_INST_LDS"]:
            if k in s:
                print(f"   {k:26s} {s[k] / wave:6.3f} of wave-cycles")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in s:
            # busy cycles summed over SIMDs (1024 on the chip) vs shader-engine cycles
            print(f"   MFMA busy                  {s['SQ_VALU_MFMA_BUSY_CYCLES'] / (1024 * s['GRBM_GUI_ACTIVE'] / 8):6.3f}")
        for k in ["SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_LDS_BANK_CONFLICT"]:
            if k in s:
                print(f"   {k:26s} {s[k]:.3e}")
        print(f"   SQ_BUSY_CYCLES {busy:.3e}  SQ_WAVE_CYCLES {wave:.3e}")


if __name__ == "__main__":
    main(*sys.argv[1:])
