"""HBM bytes of one whole training step from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) of a bench.py
command, against the step's compulsory bytes (engine.step_bytes_impl; bench.py step_roofline "impl").

The dispatches are cut into steps at the Adam launches (two per step: the sparse-form E / rel segment, then the
dense one); the last complete step is reported kernel by kernel and as a total (FETCH_SIZE x 2 per the gfx950
correction, MI355X_MICROARCH.md §HBM; KiB -> B), and merged into <outdir>/pmc_traffic.json under
"<workload>/<gemm>/n1/step".

usage: python tools/pmc_step.py <fetch_dir> <write_dir> <config> <gemm> <outdir> [features] [out.txt]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.pmc_traffic import load  # noqa: E402


def steps(df):
    df = df.sort_values("Dispatch_Id").reset_index(drop=True)
    adam = df.index[df["Kernel_Name"].str.contains("adam_kernel", regex=False)].tolist()
    ends = adam[1::2]                        # the dense-segment Adam closes a step
    cuts = [-1] + ends
    return [df.iloc[cuts[i] + 1:cuts[i + 1] + 1] for i in range(len(ends))]


def main(fetch_dir, write_dir, config, gemm, outdir, features="f32", out_txt=None):
    import bench
    from iddgcn_amd.engine import step_bytes_impl
    f, w = steps(load(fetch_dir, "FETCH_SIZE")), steps(load(write_dir, "WRITE_SIZE"))
    sf, sw = f[-1], w[-1]
    assert list(sf["Kernel_Name"]) == list(sw["Kernel_Name"]), "the two passes ran different dispatch sequences"
    rd = sf["Counter_Value"].to_numpy() * 1024 * 2
    wr = sw["Counter_Value"].to_numpy() * 1024
    cfg = bench.CONFIGS[int(config)]
    N, R, D, M = cfg["N"], cfg["R"], cfg["D"], cfg["M"]
    T = M + (M // cfg["neg_every"] if "neg_every" in cfg else M)
    eb = 2 if features == "bf16" else 4
    model, parts = step_bytes_impl(N, R, D, T, M, eb=eb, fused_sigma_tn=True,
                                   fused_tail_head=features == "bf16" and R == 8)
    lines = [f"# rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), config {config} ({cfg['name']}), {gemm}, "
             f"features {features}: HBM bytes per dispatch of the last complete step (FETCH x 2, KiB -> B); "
             f"{len(f)} steps in the trace"]
    for k, (name, dur) in enumerate(zip(sf["Kernel_Name"], sf["dur_ms"])):
        if rd[k] + wr[k] > 1e-3 * (rd.sum() + wr.sum()):
            lines.append(f"{name[:50]:50s} read {rd[k] / 1e9:8.3f} write {wr[k] / 1e9:8.3f} GB  {dur:8.3f} ms (profiled)")
    tot = float(rd.sum() + wr.sum())
    lines.append(f"step total: read {rd.sum() / 1e9:.2f} GB + write {wr.sum() / 1e9:.2f} GB = {tot / 1e9:.2f} GB; "
                 f"compulsory bytes of the formulation (engine.step_bytes_impl) {model / 1e9:.2f} GB = "
                 f"{model / tot:.3f} of the measured")
    print("\n".join(lines))
    if out_txt:
        open(out_txt, "w").write("\n".join(lines) + "\n")
    path = os.path.join(outdir, "pmc_traffic.json")
    rec = json.load(open(path)) if os.path.exists(path) else {}
    rec[f"{cfg['name']}/{gemm}/n1/step"] = {"read_bytes": float(rd.sum()), "write_bytes": float(wr.sum()),
                                            "bytes": tot, "dispatches": int(len(rd)),
                                            "step_bytes_impl": model, "impl_over_measured": model / tot}
    with open(path, "w") as fh:
        json.dump(rec, fh, indent=1, sort_keys=True)


if __name__ == "__main__":
    a = sys.argv[1:]
    main(*a[:5], *(a[5:7]))
