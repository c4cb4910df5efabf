"""HBM traffic per launch of bench.py's dominant kernel from two rocprofv3 --pmc passes.

Collection (MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE cannot share a pass; on gfx950
FETCH_SIZE reports half the bytes of wide streaming reads, so it is doubled):

  rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- python3 bench.py ...
  rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- python3 bench.py ...
  python tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write split synthetic-3 1 profiles/r01

Kernel launches are matched by symbol; the edge-level launches of a symbol are those at least half
as long as its longest launch (the same symbols also run small node-level GEMMs).  The result is
merged into <outdir>/pmc_traffic.json under "<workload>/<gemm>/n<world>/<bench kernel name>", which
bench.py reads into roofline.traffic.
"""
import glob
import json
import os
import sys

import pandas as pd

# rowgemm256_v3_kernel<NV, AUX, HAS_COEF, X3, CW, BF, PL, C4> (ABI 6 template order)
SYMBOLS = {
    # split mode: the layer-2 forward writes planes C (PL true), layer 3 does not; the backward reads planes
    "split": {"tail_fwd_gemm": "rowgemm256_v3_kernel<2, false, true, true, false, false,",
              "tail_bwd_gemm": "rowgemm256_v3_kernel<0, true, false, true, false, false,",
              "tail_dS_tn": "gemm_tn256_x3_kernel<"},
    # bf16x3 operands (ABI 7): the column-half row GEMM and the transposed-read TN
    "bf16x3": {"tail_fwd_gemm": "rowgemm256_b3_kernel<2, false, false>",
               "tail_bwd_gemm": "rowgemm256_b3_kernel<0, true, false>",
               "tail_dS_tn": "gemm_tn256_b3_kernel",
               "tail_bwd_sigma_tn": "sigma_tn_b3_kernel"},           # round 6: the fused pass (ABI 12)
    "exact": {"tail_fwd_gemm": "rowgemm256_v3_kernel<2, false, true, false, false, false, false, false>",
              "tail_bwd_gemm": "rowgemm256_v3_kernel<0, true, false, false, false, false, false, false>",
              "tail_dS_tn": "gemm_tn256_dma_kernel"},
    # the bf16-feature mode (config 5: R = 8 gathered relations, bf16 edge tables); recorded under the
    # bench's gemm key with `python tools/pmc_traffic.py ... exact synthetic-5 1 profiles/r03 bf16`
    "bf16": {"tail_fwd_gemm": "fwd_gather8_bf16_kernel",
             "tail_bwd_gemm": "rowgemm256_v3_kernel<0, true, false, true, false, true, false, false>",
             "tail_dS_tn": "gemm_tn256_bf16t_kernel",
             "tail_bwd_sigma_tn": "sigma_tn_bf16_kernel"},         # round 5: the fused pass (ABI 11)
}


def load(d, counter):
    path = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    c = pd.read_csv(path)
    c = c[c["Counter_Name"] == counter].copy()
    c["dur_ms"] = (c["End_Timestamp"] - c["Start_Timestamp"]) / 1e6
    return c.groupby(["Dispatch_Id", "Kernel_Name", "dur_ms"], as_index=False)["Counter_Value"].sum()


def edge_launches(df, sym):
    k = df[df["Kernel_Name"].str.contains(sym, regex=False)]
    return k[k["dur_ms"] >= 0.5 * k["dur_ms"].max()]


def main(fetch_dir, write_dir, gemm, workload, world, outdir, symset=None):
    f, w = load(fetch_dir, "FETCH_SIZE"), load(write_dir, "WRITE_SIZE")
    out_path = os.path.join(outdir, "pmc_traffic.json")
    rec = json.load(open(out_path)) if os.path.exists(out_path) else {}
    for name, sym in SYMBOLS[symset or gemm].items():
        fe, we = edge_launches(f, sym), edge_launches(w, sym)
        if fe.empty or we.empty:
            continue
        rd = float(fe["Counter_Value"].mean()) * 1024 * 2      # KiB, x2 gfx950 correction
        wr = float(we["Counter_Value"].mean()) * 1024
        rec[f"{workload}/{gemm}/n{world}/{name}"] = {
            "symbol": sym, "launches": int(len(fe)), "read_bytes_per_launch": rd, "write_bytes_per_launch": wr,
            "bytes_per_launch": rd + wr, "avg_ms_fetch_pass": float(fe["dur_ms"].mean()),
            "avg_ms_write_pass": float(we["dur_ms"].mean())}
        print(f"{name:14s} {sym:45s} read {rd / 1e9:7.3f} GB  write {wr / 1e9:7.3f} GB  per launch "
              f"({len(fe)} launches)")
    with open(out_path, "w") as fh:
        json.dump(rec, fh, indent=1, sort_keys=True)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3], sys.argv[4], int(sys.argv[5]), sys.argv[6],
         sys.argv[7] if len(sys.argv) > 7 else None)
