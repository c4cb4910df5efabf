"""IDDGCN training-step throughput on MI355X (BASELINE.json).

Metric: adjacency edges/s = M / (wall time of one full training step: positive forward + negative
forward + backward + Keras Adam), whole job.

Workloads (BASELINE.json configs; synthetic seeded mutation–drug graphs, reference-distribution
random init, inputs resident in HBM before the timed region):
  --config 3 (default)  100k nodes, 2 relations, 2M directed reverse-closed edges, D=256, 1:1
                        negatives (T = 4M scored edges).  With --gpus N the job is WEAK-scaled: every
                        rank owns 4M scored edges of a 2M*N-edge graph on the same 100k nodes.
  --config 4            1M nodes, 2 relations, 20M edges, D=256, T = 40M scored edges; STRONG-scaled
                        (the 40M scored edges are split over the N ranks).
  --config 5            1M nodes, 8 relations, 40M edges + 10M negatives, D=256, T = 50M; STRONG-scaled.
  --config 2            the reference's fold-0 shape (845 nodes, 4 relations, D=64), one GPU.
Multi-GPU: `--gpus N` starts N ranks itself (torch.distributed.run, one process per GPU, RCCL)
before anything touches the GPU, or joins the N ranks a launcher already started; the ranks meet in
one bucketed in-place all-reduce of the flat gradient buffer per step (parallel.BucketedAllReduce).

Also reported on the same JSON line:
  roofline      the dominant kernel's achieved HBM rate (algorithmic bytes per launch / its
                HIP-event duration inside the timed steps, events on the launch stream) vs 8 TB/s;
  cpu_baseline  the reference formulation (oracle/ref_model.py: torch-CPU fp32, per-edge GEMMs,
                A_r.E per layer, Keras BCE, Keras Adam) on this host's cores, on a bounded sample
                of the same workload (rank 0, N=1 only).
"""
import argparse
import json
import os
import socket
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

MFMA_F32_PEAK_TFLOPS = 157.3     # MI355X_MICROARCH.md, f32-input MFMA dense peak
MFMA_F16_PEAK_TFLOPS = 2500.0    # MI355X_MICROARCH.md, bf16/f16 MFMA dense peak (16x the f32 rate)
HBM_PEAK_GBS = 8000.0
GEMM_NOTE = {
    "split": "opt-in mode: D=256 GEMM operands split hi+lo fp16 (22-23 significant bits, power-of-two row/column "
             "scales), 3 f16 MFMAs per k-step, fp32 accumulation; every other kernel exact f32 "
             "(include/iddgcn.h IDDGCN_GEMM_SPLIT_F16, per call)",
    "exact": "exact f32 MFMA (v_mfma_f32_32x32x2_f32, bitwise an fmaf chain) for every GEMM, exact f32 elsewhere",
    "bf16x3": "D=256 GEMM operands split EXACTLY into three bf16 pieces (8+8+8 = 24 significant bits: every fp32 "
              "value represented without loss), the six piece products of order >= 2^-16 on bf16 MFMAs (exact "
              "products), fp32 accumulation; dropped cross terms <= 2^-23 |a*w| per product (fp32's own product "
              "rounding: 2^-24); every other kernel exact f32 (include/iddgcn.h IDDGCN_GEMM_BF16X3, per call)",
}
# the arithmetic the path computes in, per GEMM mode (the bench line's "dtype")
DTYPE = {"split": "f32 (D=256 GEMMs on split-fp16x2 operands, fp32 accumulate)", "exact": "f32", "bf16x3": "f32"}
DTYPE_BF16 = {
    "hilo": ("bf16 edge tables (x^l, do^l) with bf16 MFMA for the edge GEMMs (weights as bf16 hi+lo), fp32 node "
             "tables, accumulation and epilogues, node-level GEMMs on split-fp16 operands (perf-only mode, BASELINE "
             "config 5)"),
    "bf16": ("bf16 edge tables (x^l, do^l) with bf16 x bf16 MFMA for the edge GEMMs (every edge-GEMM operand rounded "
             "to bf16 once: weights, and the R = 8 combine's node rows and coefficients; include/iddgcn.h "
             "IDDGCN_GEMM_BF16), fp32 node tables, accumulation and epilogues, node-level GEMMs on split-fp16 "
             "operands (perf-only opt-in form of BASELINE config 5's 'bf16 features with MFMA XW': 8x the logit error of "
             "hi+lo weights at the 99% quantile, DESIGN.md)"),
}

CONFIGS = {
    2: dict(name="synthetic-fold0-shape", N=845, R=4, M=37_510, D=64, scaling="weak"),
    3: dict(name="synthetic-3", N=100_000, R=2, M=2_000_000, D=256, scaling="weak"),
    4: dict(name="synthetic-4", N=1_000_000, R=2, M=20_000_000, D=256, scaling="strong"),
    # 40M positives, 10M negatives (one per 4 positives), generated on the device
    5: dict(name="synthetic-5", N=1_000_000, R=8, M=40_000_000, D=256, scaling="strong", neg_every=4,
            features="bf16", gemm="split", edge_mfma="hilo"),
}


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(args):
    """--gpus N without a launcher: run N ranks under torch.distributed.run as a CHILD process (nothing
    has touched the GPU yet) and return its exit code; inside a launcher, check its world size."""
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None:
        if args.gpus == 1:
            return None
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
               "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.abspath(__file__),
               *sys.argv[1:]]
        return subprocess.call(cmd)
    if int(world_env) != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={world_env} ranks")
    return None


def kernel_roofline(name, N, R, D, T, gemm, avg_ms, eb=4, edge_mfma="hilo"):
    """Roofline of one edge-level GEMM launch.

    flops: 2*D^2*T algorithmic (x3 f16 MFMA instructions on the f16 peak in split mode, x6 bf16 ones in bf16x3);
    bytes (algorithmic, fp32): fwd reads x^{l-1}, writes x^l, reads W[h_e] (R per edge), t_e and the
    distinct P_r rows (R*N*D once); bwd reads do and the sigma' operand x, writes do' (the layer-2 bwd,
    "rec", rebuilds x^1 from the distinct ES1 / P^1 rows and W^1[h_e] instead of reading it); dS reads
    x and do (eb = bytes per edge-table element: 4, or 2 in the bf16-feature mode, whose GEMMs run 2 bf16
    MFMAs per k-step with hi + lo weights, 1 with bf16 weights: edge_mfma).  bound = whichever roofline time is
    larger."""
    flops = 2.0 * D * D * T
    nbytes = {"tail_fwd_gemm": 2.0 * eb * D * T + 4.0 * R * T + 4.0 * T + 4.0 * R * N * D,
              "tail_bwd_gemm": 3.0 * eb * D * T,
              "tail_bwd_rec_gemm": 2.0 * eb * D * T + 4.0 * R * T + 4.0 * T + 4.0 * (R + 1) * N * D,
              "tail_dS_tn": 2.0 * eb * D * T,
              "tail_bwd_sigma_tn": 3.0 * eb * D * T}[name]
    if name == "tail_bwd_sigma_tn" and eb == 2:
        # one pass, both GEMMs over bf16 tables: sigma' 2 bf16 products per term with hi + lo weights (1 with bf16
        # weights, edge_mfma "bf16"), the TN 1
        flops, hw_flops, peak_f = 2 * flops, (2 if edge_mfma == "bf16" else 3) * flops, MFMA_F16_PEAK_TFLOPS
    elif name == "tail_bwd_sigma_tn":
        # one pass, both GEMMs over fp32 tables in the bf16x3 mode (round 6): six bf16 products per term in each
        flops, hw_flops, peak_f = 2 * flops, 12 * flops, MFMA_F16_PEAK_TFLOPS
    elif eb == 2:
        hw_flops, peak_f = (1 if edge_mfma == "bf16" else 2) * flops, MFMA_F16_PEAK_TFLOPS
    elif gemm == "bf16x3":
        hw_flops, peak_f = 6 * flops, MFMA_F16_PEAK_TFLOPS
    elif gemm == "split":
        hw_flops, peak_f = 3 * flops, MFMA_F16_PEAK_TFLOPS
    else:
        hw_flops, peak_f = flops, MFMA_F32_PEAK_TFLOPS
    t_mfma = hw_flops / (peak_f * 1e12)
    t_hbm = nbytes / (HBM_PEAK_GBS * 1e9)
    s = avg_ms * 1e-3
    if t_hbm >= t_mfma:
        out = {"kernel": name, "bound": "hbm", "achieved": nbytes / s / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s"}
    else:
        out = {"kernel": name, "bound": "mfma", "achieved": hw_flops / s / 1e12, "peak": peak_f,
               "unit": "TFLOP/s"}
    out["frac"] = out["achieved"] / out["peak"]
    out.update({"avg_launch_ms": avg_ms, "bytes_per_launch": nbytes, "flops_per_launch": flops, "hw_flops_per_launch": hw_flops,
                "mfma_frac": hw_flops / s / 1e12 / peak_f, "hbm_frac": nbytes / s / 1e9 / HBM_PEAK_GBS})
    return out


def stream_probe(torch, dev, T, D, reps=3):
    """What this box's HBM sustains for the access mixes of the edge kernels, measured in the same
    run on one edge table (T x D fp32, capped at 4M rows): write-only (fill), read+write 1:1 (copy),
    read-only (sum).  Context for roofline.frac, whose peak is the 8 TB/s vendor figure."""
    T = min(T, 4_000_000)
    a = torch.empty(T, D, dtype=torch.float32, device=dev)
    b = torch.empty_like(a)
    out = {}
    for name, fn, nbytes in (("fill", lambda: a.fill_(1.0), a.numel() * 4),
                             ("copy", lambda: b.copy_(a), 2 * a.numel() * 4),
                             ("read", lambda: a.sum(), a.numel() * 4)):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        out[name] = nbytes / (e0.elapsed_time(e1) / reps * 1e-3) / 1e9
    del a, b
    return out


def pmc_record(key):
    """An entry of the NEWEST committed rocprofv3 PMC summary (profiles/rNN/pmc_traffic.json of the latest round,
    written by tools/pmc_traffic.py / tools/pmc_step.py: FETCH_SIZE x2 per the gfx950 correction + WRITE_SIZE,
    separate --pmc passes), or (None, None).  Older rounds' files are not consulted: their kernels may have changed."""
    import glob
    paths = sorted(glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]", "pmc_traffic.json")))
    if not paths:
        return None, None
    with open(paths[-1]) as f:
        rec = json.load(f)
    return rec.get(key), os.path.relpath(paths[-1], ROOT)


def pmc_traffic(kernel, gemm, workload, world):
    """HBM bytes per launch of `kernel` of the same bench command (pmc_record), or None."""
    r, path = pmc_record(f"{workload}/{gemm}/n{world}/{kernel}")
    return (r["bytes_per_launch"], path) if r else (None, None)


def workload_bytes(cid, world, features):
    """Upper estimate of one rank's device memory for a workload (engine.Workspace, graph, parameters with
    gradients and Adam moments, + the device graph build's sort buffers), for the multi-rank fit check."""
    cfg = CONFIGS[cid]
    N, R, D = cfg["N"], cfg["R"], cfg["D"]
    M = cfg["M"] * (world if cfg["scaling"] == "weak" else 1)
    T = M + M // cfg.get("neg_every", 1)
    Tr = -(-T // world)
    eb = 2 if features == "bf16" else 4
    edge = 3 * Tr * D * eb + Tr * (4 * 4 + 8 + 4 + 4 * 4 * R + 8)
    node = 4 * N * D * (6 * R + 7) + 4 * N * R * 8
    params = 4 * 4 * (N * D + 3 * (R + 1) * D * D + R * D)
    graph = 32 * M + 40 * T
    return int(1.15 * (edge + node + params + graph)) + (2 << 30)


def reference_init(np, N, R, D, seed):
    """Reference-distribution init (IDDGCN.py:25-58, 92-101, 221-224)."""
    rng = np.random.default_rng(seed)
    p = {"E": rng.random((N, D), dtype=np.float32)}
    lim = np.sqrt(6.0 / (D + R))
    for l in (1, 2, 3):
        p[f"K{l}"] = rng.standard_normal((R, D, D), dtype=np.float32)
        p[f"S{l}"] = rng.standard_normal((D, D), dtype=np.float32)
        p[f"Wa{l}"] = rng.uniform(-lim, lim, (D, R)).astype(np.float32)
        p[f"ba{l}"] = np.zeros(R, np.float32)
    p["rel"] = rng.standard_normal((R, D), dtype=np.float32)
    return p


FOLD0_REFERENCE_AUC = 0.9072     # the reference's eval ROC-AUC of fold 0 with its bundled trained weights


def fold0_auc(dev, epochs=5000):
    """The metric's second part, "AUC vs reference on fold-0" (BASELINE.json): the reference's fold-0 split and
    weights, converted once into tests/golden/ (data fixtures: fold0_data.npz, weights_fold0.npz), through the product
    API (get_IDDGCN_Model -> predict / fit: IDDGCN_eval.py:35-122, IDDGCN.py:287-412).  Two numbers: the eval AUC with
    the reference's bundled trained weights, and the eval AUC after training fold 0 from TF 2.7's replayed initial
    weights for the reference's 5000 epochs (fit() on the kernels, HIP-graph replay), each beside the reference's
    0.9072; plus the training time."""
    import numpy as np
    from sklearn.metrics import roc_auc_score
    from iddgcn_amd import Adam, BinaryCrossentropy, get_IDDGCN_Model
    from iddgcn_amd.graph import get_adj_mats
    n_ent, n_rel, dim = 845, 4, 64
    gold = os.path.join(ROOT, "tests", "golden")
    d = np.load(os.path.join(gold, "fold0_data.npz"))
    adj_eval = get_adj_mats(np.concatenate([d["X_train"], d["X_test"]]), n_ent, n_rel)
    Xt = np.concatenate([d["X_test"], d["neg_X_test"]])[None]
    y = np.concatenate([np.ones(len(d["X_test"])), np.zeros(len(d["neg_X_test"]))])

    def auc(model):
        p = model.predict(x=[np.arange(n_ent)[None], Xt[:, :, 0], Xt[:, :, 1], Xt[:, :, 2], adj_eval])[0]
        return float(roc_auc_score(y, p))

    ref_model = get_IDDGCN_Model(n_ent, n_rel, dim, dim, 89, None, 0, 0)
    ref_model.load_weights(os.path.join(gold, "weights_fold0.npz"))
    a_bundled = auc(ref_model)
    model = get_IDDGCN_Model(n_ent, n_rel, dim, dim, 89, None, 0, 0, init="tf27")
    model.neg_triples = d["X_train_neg"][None]
    model.compile(loss=BinaryCrossentropy(), optimizer=Adam(learning_rate=0.001))
    X = d["X_train"][None]
    import torch
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    model.fit(x=[np.arange(n_ent)[None], X[:, :, 0], X[:, :, 1], X[:, :, 2], get_adj_mats(d["X_train"], n_ent, n_rel)],
              y=np.ones((1, X.shape[1])), epochs=epochs, batch_size=100, verbose=0)
    torch.cuda.synchronize()
    fit_s = time.perf_counter() - t0
    a_trained = auc(model)
    return {"reference": FOLD0_REFERENCE_AUC, "bundled_weights": a_bundled,
            "trained_from_replayed_init": a_trained, "epochs": epochs, "fit_s": fit_s,
            "delta_bundled": a_bundled - FOLD0_REFERENCE_AUC, "delta_trained": a_trained - FOLD0_REFERENCE_AUC,
            "within_0.001": abs(a_bundled - FOLD0_REFERENCE_AUC) <= 1e-3 and abs(a_trained - FOLD0_REFERENCE_AUC) <= 1e-3,
            "source": "tests/golden/fold0_data.npz + weights_fold0.npz (the reference's bundled fold-0 files, converted)"}


def cpu_model():
    """The host CPU's model name (/proc/cpuinfo), for the cpu_baseline record (core count and CPU
    model next to every CPU number)."""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cgroup_cpu_quota():
    """CPUs granted by the cgroup v2 (cpu.max) or v1 (cfs quota / period) CPU controller, rounded up; None if
    unlimited or unreadable."""
    import math
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()[:2]
        return None if q == "max" else max(1, math.ceil(int(q) / int(p)))
    except (OSError, ValueError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            q = int(f.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            p = int(f.read())
        return None if q <= 0 else max(1, math.ceil(q / p))
    except (OSError, ValueError):
        return None


def cpu_baseline(cfg, frac=0.05, min_steps=3, budget_s=60.0):
    """The reference formulation on the host cores (one full step: pos + neg forward, autograd backward,
    Keras Adam), on a bounded sample of the same workload: the same N, D, R and a `frac` share of its
    adjacency edges (and as many negatives).  The reference formulation's cost is linear in the edges
    (per-edge GEMMs, SpMM per layer), so edges/s on the sample is the full step's rate (its per-layer dense
    N x D SpMM outputs are a fixed cost that a smaller sample weighs more: the sample's rate is a lower bound
    of the full workload's).  Protocol: one warm-up step, then the median of `min_steps` timed
    steps (more while the budget allows)."""
    import numpy as np
    import torch
    from oracle.ref_model import KerasAdam, adj_to_torch, keras_bce, model_forward, to_torch_params
    from oracle.ref_utils import get_adj_coo
    from iddgcn_amd.utils import synthetic_graph
    N, R, D = cfg["N"], cfg["R"], cfg["D"]
    # every core this process may run on (torch.set_num_threads(os.cpu_count())), bounded by what the
    # lease grants: the affinity mask and the cgroup CPU quota (the GPU box shows the whole host's CPUs in both
    # os.cpu_count() and the mask, and grants a 16-CPU share), all counts on the record
    affinity = len(os.sched_getaffinity(0))
    quota = cgroup_cpu_quota()
    usable = min(affinity, quota) if quota else affinity
    threads_before = torch.get_num_threads()
    torch.set_num_threads(usable)
    threads = torch.get_num_threads()

    def make(M_s):
        pos, neg = synthetic_graph(N, R, M_s, seed=11)
        params = {k: v for k, v in reference_init(np, N, R, D, 89).items()}
        return pos, neg, params, adj_to_torch(get_adj_coo(pos, N, R), N, torch.float32), KerasAdam()

    def step(pos, neg, params, adj, opt):
        P = to_torch_params(params, torch.float32)
        y_pos = model_forward(P, pos[:, 0], pos[:, 1], pos[:, 2], adj)
        y_neg = model_forward(P, neg[:, 0], neg[:, 1], neg[:, 2], adj)
        y = torch.cat([y_pos, y_neg])
        loss = keras_bce(torch.cat([torch.ones_like(y_pos), torch.zeros_like(y_neg)]), y) / N
        keys = [k for k in P if P[k].requires_grad]
        grads = torch.autograd.grad(loss, [P[k] for k in keys])
        return opt.step(params, {k: g.numpy() for k, g in zip(keys, grads)}, dtype=np.float32)

    M_s = max(1, int(round(cfg["M"] * frac)))
    pos, neg, params, adj, opt = make(M_s)
    params = step(pos, neg, params, adj, opt)           # warm-up (thread pool, allocator) on the same sample
    times = []
    while True:
        t0 = time.perf_counter()
        params = step(pos, neg, params, adj, opt)
        times.append(time.perf_counter() - t0)
        if len(times) >= min_steps and (len(times) >= 5 or sum(times) + times[-1] > budget_s):
            break
    t = statistics.median(times)
    torch.set_num_threads(threads_before)
    return {"value": M_s / t, "unit": "adjacency edges/s", "cores": threads, "kind": "port",
            "host_cpu_count": os.cpu_count(), "cpus_in_affinity_mask": affinity,
            "cgroup_cpu_quota": quota,
            "torch_threads_default": threads_before, "cpu_model": cpu_model(),
            "fraction_of_workload": M_s / cfg["M"], "step_s": times,
            "scored_edges_per_s": 2 * M_s / t,
            "sample": (f"oracle/ref_model.py reference formulation (torch-CPU fp32: per-edge GEMMs, A_r.E per layer, "
                       f"Keras BCE, autograd backward, Keras Adam), N={N} D={D} R={R}, {M_s} of the workload's "
                       f"{cfg['M']} adjacency edges ({100 * M_s / cfg['M']:.0f}%) + {M_s} negatives; median of "
                       f"{len(times)} steps after a warm-up step, {t:.2f} s/step, {threads} torch threads "
                       f"(torch.set_num_threads: {affinity} CPUs in the affinity mask, cgroup quota {quota} CPUs) on a "
                       f"{os.cpu_count()}-CPU host ({cpu_model()})")}


def step_roofline(N, R, D, T, M, gemm, features, ms_per_step, edge_mfma="hilo", fused_sigma_tn=True,
                  fused_tail_head=False):
    """Whole-step roofline of one rank's step (round 6: a lower bound of THIS formulation).

    impl: engine.step_bytes_impl's parts (the compulsory HBM bytes and D x D GEMM work of each stage of the
      implemented step: tail-sorted gathers read each distinct node row once, SpMM gathers from tables beyond the
      256 MiB Infinity Cache once per stored entry, small random-order rows one 128-B line each); each part priced at
      the larger of its MFMA time (the MFMA products this mode issues per flop, on that MFMA's dense peak) and its
      HBM time at 8 TB/s, summed over the parts.  T_roof <= the measured step by construction, frac = T_roof / T.
    survey_formula: SURVEY §8(d)'s W_gemm / P + Q_hbm / BW as written (Q_hbm charges every scored edge R gathered
      P_r rows per layer, 8·L·R·T·D; W_gemm on the f32 peak) and with W_gemm on this mode's MFMA peak: kept for
      comparison, NOT a lower bound of this formulation (its ratio to the measured step can exceed 1)."""
    from iddgcn_amd.engine import step_bytes, step_bytes_impl, step_flops
    W = float(step_flops(N, R, D, T, M))
    Q = float(step_bytes(N, R, D, T, M))
    if features == "bf16":          # "for bf16, use 2.5 PFLOP/s and halve the D-terms"
        Q = Q - 0.5 * (40.0 * T * D + 8.0 * 3 * R * T * D)
    # MFMA products per algorithmic flop and their peak, for the edge-level and the node-level GEMMs of this mode
    node = {"exact": (1, MFMA_F32_PEAK_TFLOPS), "split": (3, MFMA_F16_PEAK_TFLOPS),
            "bf16x3": (6, MFMA_F16_PEAK_TFLOPS)}[gemm]
    edge = node
    if features == "bf16":          # bf16 tables: x·S and sigma' 2 products (hi + lo weights) or 1, the dS TN 1
        edge = ((1.0 if edge_mfma == "bf16" else 1.5), MFMA_F16_PEAK_TFLOPS)
    Qi, parts = step_bytes_impl(N, R, D, T, M, eb=2 if features == "bf16" else 4, fused_sigma_tn=fused_sigma_tn,
                                fused_tail_head=fused_tail_head)
    t_parts = {}
    for name, (nbytes, flop, kind) in parts.items():
        hw, peak = {"edge": edge, "node": node}.get(kind, (0, 1.0))
        t_parts[name] = max(hw * flop / (peak * 1e12), nbytes / (HBM_PEAK_GBS * 1e9)) * 1e3
    t_impl = sum(t_parts.values())
    t_hbm = Q / (HBM_PEAK_GBS * 1e9) * 1e3
    t_f32 = W / (MFMA_F32_PEAK_TFLOPS * 1e12) * 1e3
    hw_mode = node[0] if features != "bf16" else edge[0]
    t_mode = hw_mode * W / (node[1] * 1e12) * 1e3
    return {"impl": {"Q_hbm_bytes": Qi, "W_gemm_flop": sum(v[1] for v in parts.values()), "t_roof_ms": t_impl,
                     "frac": t_impl / ms_per_step, "t_hbm_ms": Qi / (HBM_PEAK_GBS * 1e9) * 1e3,
                     "parts_ms": {k: round(v, 4) for k, v in t_parts.items()},
                     "parts_GB": {k: round(v[0] / 1e9, 3) for k, v in parts.items()},
                     "fused_sigma_tn": bool(fused_sigma_tn), "fused_tail_head": bool(fused_tail_head)},
            "survey_formula": {"W_gemm_flop": W, "Q_hbm_bytes": Q, "t_hbm_ms": t_hbm,
                               "f32_peak": {"t_mfma_ms": t_f32, "t_roof_ms": t_f32 + t_hbm,
                                            "ratio_to_measured": (t_f32 + t_hbm) / ms_per_step},
                               "mode_peak": {"mfma_products_per_flop": hw_mode, "t_mfma_ms": t_mode,
                                             "t_roof_ms": t_mode + t_hbm, "ratio_to_measured": (t_mode + t_hbm) / ms_per_step},
                               "note": "SURVEY §8(d) as written; not a lower bound of this formulation"}}


def rank_consistency(buf):
    """After the timed steps: the largest |params - rank 0's params| over all ranks (0.0 when every rank holds
    bitwise the same parameters, as the replicated Adam on all-reduced gradients must).  ``buf``: the rank's flat
    parameter buffer (FlatParams.buf) on its GPU."""
    import torch.distributed as dist
    ref = buf.clone()
    dist.broadcast(ref, 0)
    d = (buf - ref).abs().max().reshape(1)
    if dist.get_backend() != "nccl":
        d = d.cpu()
    dist.all_reduce(d, op=dist.ReduceOp.MAX)
    del ref
    return float(d.item())


def run_workload(cid, args, world, rank, dev, gemm, other_mode, probe_kernels=True, shard=None, steps=None,
                 warmup=None):
    """Build one workload on the GPU, time W + K training steps, return the bench-line fields."""
    import numpy as np
    import torch
    import torch.distributed as dist
    from iddgcn_amd.engine import Engine, FlatParams, KerasAdam
    from iddgcn_amd.graph import get_adj_mats
    from iddgcn_amd.parallel import BucketedAllReduce, RelationShard, shard_range
    from iddgcn_amd.utils import synthetic_graph

    cfg = CONFIGS[cid]
    N, R, D = cfg["N"], cfg["R"], cfg["D"]
    # config 5 is the bf16-feature throughput mode: its node-level GEMMs take split-fp16 operands too
    gemm = cfg.get("gemm", gemm) if (args.features or cfg.get("features", "f32")) == "bf16" else gemm
    shard = args.shard if shard is None else shard
    steps = args.steps if steps is None else steps
    warmup = args.warmup if warmup is None else warmup
    weak = cfg["scaling"] == "weak"
    M = cfg["M"] * world if weak else cfg["M"]            # weak: per-GPU work fixed
    pos, neg = synthetic_graph(N, R, M, seed=0)           # identical on every rank (seeded)
    if cfg.get("neg_every", 1) > 1:
        # one negative per neg_every positives, drawn ON THE DEVICE with the reference's recipe
        # (utils1.py:646-655, MT19937 stream bit-exact to numpy's, csrc/sampling.hip)
        from iddgcn_amd.sampling import negative_samples
        neg = negative_samples(pos[::cfg["neg_every"]], N, 89, device=dev)
    T = len(pos) + len(neg)
    npos = len(pos)
    cuts = None
    if shard == "node" and world > 1:
        # node-row partitioning: rank k owns a contiguous node range (balanced by tail edges + node work) and the
        # scored edges whose tail it owns (parallel.NodeShard)
        from iddgcn_amd.parallel import node_ranges, node_row_weight, node_shard_triples
        cuts = node_ranges(np.bincount(np.concatenate([pos[:, 2], neg[:, 2]]), minlength=N), world,
                           node_weight=node_row_weight(R, args.features or cfg.get("features", "f32")))
        tri, lab = node_shard_triples(np.concatenate([pos, neg]),
                                      np.concatenate([np.ones(npos, np.float32), np.zeros(len(neg), np.float32)]),
                                      cuts, rank)
    else:
        lo, hi = shard_range(T, rank, world)              # this rank's contiguous shard (pos ++ neg)
        tri = np.concatenate([pos[lo:min(hi, npos)], neg[max(lo - npos, 0):max(hi - npos, 0)]])
        lab = np.concatenate([np.ones(max(0, min(hi, npos) - lo), np.float32),
                              np.zeros(max(0, hi - max(lo, npos)), np.float32)])
    feat = args.features or cfg.get("features", "f32")
    emfma = cfg.get("edge_mfma", "hilo") if feat == "bf16" else "hilo"
    eng = Engine(N, R, D, dev, gemm=gemm, features=feat, planes=not args.no_planes, edge_mfma=emfma)
    eng.overlap = args.overlap
    adj = get_adj_mats(pos, N, R, device=dev)            # device graph build (bit-identical to the host's)
    ed = eng.edges(tri, lab)
    del pos, neg, tri, lab
    P, G = FlatParams(N, R, D, dev), FlatParams(N, R, D, dev)
    init = reference_init(np, N, R, D, 89)
    comm = BucketedAllReduce() if world > 1 else None
    if cuts is not None:
        from iddgcn_amd.parallel import NodeShard
        eng.row_shard = NodeShard(cuts)          # node rows split over the ranks, scored edges by tail
        eng.overlap_e_gather = True              # the E all-gather travels into the next step (finished below)
        eng.split_e_collectives = bool(getattr(args, "split_e", False))   # opt-in: per-owner E pieces (round 6)
    elif shard == "relation" and world > 1:
        eng.node_shard = RelationShard(R, N)     # SURVEY §8(e) alternative: node tables split by relation
    elif shard == "spmm" and world > 1:
        eng.spmm_shard = RelationShard(R, N)     # row-partitioned SpMMs, node GEMMs replicated

    def timed_run(mode, probe, edge_mfma=emfma):
        """W warm-up steps, then K timed steps between barriers + synchronize; max over ranks."""
        eng.gemm = mode
        eng.edge_mfma = edge_mfma
        P.load(init)                       # every mode starts from the same parameters
        opt = KerasAdam(P)
        for _ in range(warmup):
            eng.train_step(P, G, opt, adj, ed, t_global=T, comm=comm)
        eng.finish_pending()
        torch.cuda.synchronize()
        eng.probe = {} if probe else None
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            loss = eng.train_step(P, G, opt, adj, ed, t_global=T, comm=comm)
        eng.finish_pending()               # node rows: the last step's all-gather of E (its work, inside the timing)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([elapsed], device=dev if dist.get_backend() == "nccl" else "cpu")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t.item())
        probe_out, eng.probe = eng.probe, None
        return elapsed, float(loss.item()) / T, probe_out

    elapsed, loss_val, probe = timed_run(gemm, probe_kernels)
    consist = rank_consistency(P.buf) if world > 1 else None
    out = {"value": M / (elapsed / steps), "ms_per_step": elapsed / steps * 1e3,
           "scaling": cfg["scaling"], "dtype": DTYPE_BF16[emfma] if feat == "bf16" else DTYPE[gemm],
           "gemm_operands": GEMM_NOTE[gemm] + (f"; edge GEMMs on bf16 edge tables, edge_mfma={emfma}"
                                               if feat == "bf16" else ""),
           "config": {"workload": cfg["name"], "num_nodes": N, "num_relations": R, "adjacency_edges": M,
                      "scored_edges": T, "scored_edges_per_gpu": ed.T, "feat_dim": D,
                      "parallelism": (f"node-rows{world}" + ("+split-e" if eng.split_e_collectives else "")
                                      if eng.row_shard else f"edge-dp{world}")
                      + ("+relation-sharded-nodes" if eng.node_shard else "")
                      + ("+row-partitioned-spmm" if eng.spmm_shard else ""),
                      "gemm": gemm, "features": feat, **({"edge_mfma": emfma} if feat == "bf16" else {})},
           "scored_edges_per_s": T / (elapsed / steps), "loss": loss_val, "steps": steps, "warmup": warmup,
           "step_roofline": step_roofline(N, R, D, ed.T, M, gemm, feat, elapsed / steps * 1e3, edge_mfma=emfma,
                                          fused_sigma_tn=eng.sigma_tn_fused,
                                          fused_tail_head=eng.fuse_tail_head and feat == "bf16" and R == 8 and D == 256)}
    step_pmc, step_pmc_src = pmc_record(f"{cfg['name']}/{gemm}/n{world}/step")
    if step_pmc:        # the measured HBM bytes of a whole step (tools/pmc_step.py) beside the compulsory count
        out["step_roofline"]["impl"].update({"pmc_step_bytes": step_pmc["bytes"], "pmc_source": step_pmc_src,
                                             "impl_over_pmc": out["step_roofline"]["impl"]["Q_hbm_bytes"] /
                                             step_pmc["bytes"]})
    if world > 1:
        out["ranks_consistent"] = consist == 0.0
        out["params_max_abs_diff_vs_rank0"] = consist
        # the RCCL calls of the multi-rank branches (NodeShard's padded all_gather / reduce_scatter incl. the node-row
        # E ownership, BucketedAllReduce's asynchronous in-place buckets, RelationShard's collectives, this consistency
        # check) have executed on RCCL at world size 1 on a builder box (tests/test_gpu_rccl.py: bitwise the gloo and
        # the communicator-free steps; profiles/r05/gpu_tests_r05b.txt) and over gloo at world 2-3; never with more
        # than one GPU before a multi-GPU driver run (every builder box has one GPU)
        out["rccl_paths_verified_before_this_run"] = {"rccl_world1_on_one_gpu": True, "gloo_world2_3": True,
                                                      "rccl_multi_gpu": False}
    if other_mode and feat == "f32":
        mode2 = "exact" if gemm != "exact" else "bf16x3"
        el2, loss2, _ = timed_run(mode2, False)
        out["other_gemm_mode"] = {"gemm": mode2, "dtype": DTYPE[mode2], "value": M / (el2 / steps),
                                  "ms_per_step": el2 / steps * 1e3, "loss": loss2}
    if other_mode and feat == "bf16":
        # the other operand form of the bf16 edge GEMMs on the same engine and inputs: weights as bf16 hi + lo
        em2 = "hilo" if emfma == "bf16" else "bf16"
        el2, loss2, _ = timed_run(gemm, False, edge_mfma=em2)
        out["other_edge_mfma"] = {"edge_mfma": em2, "dtype": DTYPE_BF16[em2], "value": M / (el2 / steps),
                                  "ms_per_step": el2 / steps * 1e3, "loss": loss2}
    if probe:
        # dominant kernel: largest total event time inside the timed steps; its roofline is the larger
        # of the MFMA time (hardware MFMA work on the mode's peak) and the HBM time (algorithmic bytes)
        kt = {k: [a.elapsed_time(b) for a, b in v] for k, v in probe.items()}
        dom = max(kt, key=lambda k: sum(kt[k]))
        rl = kernel_roofline(dom, N, R, D, ed.T, gemm, statistics.mean(kt[dom]), eb=2 if feat == "bf16" else 4,
                             edge_mfma=emfma)
        rl["traffic"], rl["traffic_source"] = pmc_traffic(dom, gemm, cfg["name"], world)
        rl["box_stream_GBs"] = stream_probe(torch, dev, ed.T, D)
        out["kernel_ms_per_step"] = {k: sum(v) / steps for k, v in kt.items()}
        out["roofline"] = rl
    del eng, adj, ed, P, G
    torch.cuda.empty_cache()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", type=int, default=3, choices=sorted(CONFIGS))
    ap.add_argument("--also", nargs="*", default=None,
                    help="further workloads timed in the same run (min(steps, 5) steps, 1 warm-up), reported "
                         "under 'also': config ids (with the run's --shard), 'Nn' = config N node-row partitioned, "
                         "'Ne' = edge-partitioned, 'Nr' = with relation-sharded node tables, 'Ns' = with "
                         "row-partitioned SpMMs; default 4 5 (BASELINE configs 4 and 5), plus 4e with more than one "
                         "GPU; none to skip")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-fold0-auc", action="store_true",
                    help="skip the metric's second part: the fold-0 eval AUC (bundled weights, and trained from scratch)")
    ap.add_argument("--no-planes", action="store_true",
                    help="fp32 tail tables x^1, x^2 instead of the pre-split planes form (A/B)")
    ap.add_argument("--shard", default=None, choices=["edge", "node", "relation", "spmm"],
                    help="multi-GPU: node-row partitioning (the default with more than one GPU: node tables split by "
                         "row range, scored edges by tail, parallel.NodeShard), edge partitioning only (node work "
                         "replicated), also relation-sharded node tables, or also row-partitioned SpMMs (A_r E "
                         "all-gathered, dAE reduce-scattered; node GEMMs replicated)")
    ap.add_argument("--split-e", action="store_true",
                    help="node rows: E as one broadcast per owner and A_r E as one SpMM per source owner, dE reduced "
                         "to each owner as the transposed SpMM writes it (Engine.split_e_collectives; opt-in)")
    ap.add_argument("--features", default=None, choices=["f32", "bf16"],
                    help="edge-table storage (default: the config's; bf16 = config 5's perf-only mode)")
    ap.add_argument("--gemm", default="bf16x3", choices=["exact", "bf16x3", "split"],
                    help="operand precision of the D=256 MFMA GEMMs: bf16x3 (the headline: fp32 operands split "
                         "exactly into three bf16 pieces, fp32 products and sums on bf16 MFMAs), exact (f32 MFMA, "
                         "bitwise an fmaf chain; timed too, under other_gemm_mode) or the opt-in split-fp16 operands")
    ap.add_argument("--no-other-mode", action="store_true", help="skip timing the other GEMM mode")
    ap.add_argument("--overlap", action="store_true",
                    help="backward: layer-2/3 tail reductions on a side stream beside the dS TN (A/B)")
    args = ap.parse_args()
    if args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if args.shard is None:
        # node-row partitioning beats edge partitioning at every config once there is more than one rank: the node
        # work is divided instead of replicated (measured per-rank compute, collective volumes)
        args.shard = "node" if args.gpus > 1 or int(os.environ.get("WORLD_SIZE", "1")) > 1 else "edge"
    rc = launch_ranks(args)
    if rc is not None:
        sys.exit(rc)

    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # RCCL over xGMI; IDDGCN_DIST_BACKEND=gloo rehearses the multi-rank path with several ranks sharing
    # fewer GPUs (host-staged buckets, tests and 1-GPU boxes only)
    backend = os.environ.get("IDDGCN_DIST_BACKEND", "nccl")
    if backend == "gloo":
        local = local % torch.cuda.device_count()
    if world > 1:
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", local)

    main_out = run_workload(args.config, args, world, rank, dev, args.gemm, not args.no_other_mode)
    main_out.pop("steps"), main_out.pop("warmup")
    result = {
        "metric": "adjacency edges/s per IDDGCN training step (pos fwd + neg fwd + bwd + Adam)",
        "value": main_out.pop("value"),
        "unit": "edges/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": main_out.pop("ms_per_step"),
        "higher_is_better": True,
        "scaling": main_out.pop("scaling"),
        "vs_baseline": None,
        "dtype": main_out.pop("dtype"),
        "data": "synthetic (seeded mutation-drug graph, reference-distribution random init)",
        "config": main_out.pop("config"),
    }
    result.update(main_out)
    if world > 1:
        result["world"] = world
        result["backend"] = dist.get_backend()
    also = []
    todo = (["4", "5"] + (["4e"] if world > 1 else [])) if args.also is None else \
        [a for a in args.also if a != "none"]
    for item in todo:
        cid = int(item.rstrip("rsne"))
        shard = {"r": "relation", "s": "spmm", "n": "node", "e": "edge"}.get(item[-1], args.shard)
        if cid == args.config and shard == args.shard:
            continue
        name = CONFIGS[cid]["name"] + {"relation": "+relation-sharded", "spmm": "+row-partitioned-spmm",
                                       "node": "+node-rows" if world > 1 else ""}.get(shard, "")
        if world > 1:
            # ranks decide TOGETHER whether the workload fits (a rank that ran out of memory alone would leave the
            # others waiting in a collective), then run it without recovery: any failure ends every rank
            torch.cuda.empty_cache()
            need = workload_bytes(cid, world, args.features or CONFIGS[cid].get("features", "f32"))
            fits = torch.tensor([1.0 if torch.cuda.mem_get_info(dev)[0] >= need else 0.0], device=dev)
            if dist.get_backend() != "nccl":
                fits = fits.cpu()
            dist.all_reduce(fits, op=dist.ReduceOp.MIN)
            if fits.item() < 1.0:
                also.append({"config": {"workload": name}, "skipped": f"does not fit every rank ({need / 2**30:.0f} GiB)"})
                continue
            also.append(run_workload(cid, args, world, rank, dev, args.gemm, False, shard=shard,
                                     steps=min(args.steps, 5), warmup=1))
            continue
        try:
            # config 5 (bf16 edge tables) also times the edge GEMMs' other operand form on the same engine
            o = run_workload(cid, args, world, rank, dev, args.gemm,
                             CONFIGS[cid].get("features") == "bf16" and not args.no_other_mode, shard=shard,
                             steps=min(args.steps, 5), warmup=1)
        except torch.OutOfMemoryError as e:      # one process: a secondary workload never costs the headline line
            torch.cuda.empty_cache()
            o = {"config": {"workload": name}, "error": f"out of memory: {e}"[:300]}
        except Exception as e:                   # nor does any other failure of one (reported, not raised)
            torch.cuda.synchronize()
            torch.cuda.empty_cache()
            o = {"config": {"workload": name}, "error": f"{type(e).__name__}: {e}"[:300]}
        also.append(o)
    if also:
        result["also"] = also
    if world == 1 and not args.no_fold0_auc:       # (at N > 1, fit() would shard fold 0 over the ranks: N = 1 only)
        try:
            result["fold0_auc"] = fold0_auc(dev)
        except Exception as e:                   # reported, never costs the bench line
            result["fold0_auc"] = {"error": f"{type(e).__name__}: {e}"[:300]}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(CONFIGS[args.config])
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
