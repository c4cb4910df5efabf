"""IDDGCN training-step throughput on MI355X (BASELINE.json).

Metric: adjacency edges/s = M / (wall time of one full training step:
positive forward + negative forward + backward + Keras Adam), whole job.

Workload (default, N=1 GPU): BASELINE.json configs[2] — synthetic mutation–drug
graph, 100,000 nodes, 2 relations, 2,000,000 directed (reverse-closed) edges,
feature dim 256, fp32, 1:1 negatives (B_pos = B_neg = 2M, T = 4M scored edges).
With --gpus N (one process per GPU, torchrun, RCCL) the job is weak-scaled:
M = 2M x N edges on the same 100k nodes, every rank owns 4M scored edges and
the ranks meet in ONE all-reduce of the flat gradient buffer per step.

Also reported, on the same JSON line:
  roofline      the dominant kernel's achieved FLOP rate (algorithmic flops per
                launch / its HIP-event duration inside the timed steps) against
                the f32 MFMA peak;
  cpu_baseline  the reference formulation (oracle/ref_model.py, torch-CPU fp32,
                per-edge GEMMs, IDDGCN.py:60-79) on this host's cores, on a
                bounded sample of the same workload (rank 0, N=1 only).
"""
import argparse
import json
import os
import statistics
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from iddgcn_amd.engine import Engine, FlatParams, KerasAdam  # noqa: E402
from iddgcn_amd.graph import get_adj_mats  # noqa: E402
from iddgcn_amd.parallel import GradAllReduce  # noqa: E402
from iddgcn_amd.utils import synthetic_graph  # noqa: E402

MFMA_F32_PEAK_TFLOPS = 157.3     # MI355X_MICROARCH.md, f32-input MFMA dense peak
HBM_PEAK_GBS = 8000.0

CONFIGS = {
    3: dict(name="synthetic-3", N=100_000, R=2, M=2_000_000, D=256),
    2: dict(name="synthetic-fold0-shape", N=845, R=4, M=37_510, D=64),
}


def reference_init(N, R, D, seed):
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


def cpu_baseline(cfg, budget_s=25.0):
    """Reference formulation on the host cores, bounded sample of the same workload."""
    from oracle.ref_model import KerasAdam as RefAdam  # noqa: F401  (same step as the reference)
    from oracle.ref_model import adj_to_torch, keras_bce, model_forward, to_torch_params
    from oracle.ref_utils import get_adj_coo
    N, R, D = cfg["N"], cfg["R"], cfg["D"]
    M_s = 40_000 if cfg["M"] > 40_000 else cfg["M"]
    pos, neg = synthetic_graph(N, R, M_s, seed=11)
    params = reference_init(N, R, D, 89)
    adj = adj_to_torch(get_adj_coo(pos, N, R), N, torch.float32)
    threads = torch.get_num_threads()

    def step():
        P = to_torch_params(params, torch.float32)
        y_pos = model_forward(P, pos[:, 0], pos[:, 1], pos[:, 2], adj)
        y_neg = model_forward(P, neg[:, 0], neg[:, 1], neg[:, 2], adj)
        y = torch.cat([y_pos, y_neg])
        loss = keras_bce(torch.cat([torch.ones_like(y_pos), torch.zeros_like(y_neg)]), y) / N
        keys = [k for k in P if P[k].requires_grad]
        grads = torch.autograd.grad(loss, [P[k] for k in keys])
        with torch.no_grad():  # Adam-sized elementwise update over every parameter
            for k, g in zip(keys, grads):
                P[k].sub_(1e-3 * g / (g.abs() + 1e-7))

    t0 = time.perf_counter()
    step()
    first = time.perf_counter() - t0
    times = []
    n = max(1, min(3, int(budget_s / max(first, 1e-3))))
    for _ in range(n):
        t0 = time.perf_counter()
        step()
        times.append(time.perf_counter() - t0)
    t = statistics.median(times)
    return {"value": M_s / t, "unit": "adjacency edges/s", "cores": threads, "kind": "port",
            "sample": (f"oracle/ref_model.py reference formulation (torch-CPU fp32, per-edge GEMMs, A_r.E per layer), "
                       f"N={N} D={D} R={R}, M={M_s} edges + {M_s} negatives (bounded sample of the workload); "
                       f"median of {n} steps after 1 warm-up, {t:.2f} s/step")}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", type=int, default=3, choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    cfg = CONFIGS[args.config]
    N, R, D = cfg["N"], cfg["R"], cfg["D"]
    M = cfg["M"] * world                                  # weak scaling: M per GPU fixed

    pos, neg = synthetic_graph(N, R, M, seed=0)           # identical on every rank (seeded)
    adj_mats = get_adj_mats(pos, N, R)
    T = len(pos) + len(neg)
    # this rank's contiguous shard of the scored edges (positives ++ negatives)
    lo, hi = rank * T // world, (rank + 1) * T // world
    tri = np.concatenate([pos, neg])[lo:hi]
    lab = np.concatenate([np.ones(len(pos), np.float32), np.zeros(len(neg), np.float32)])[lo:hi]

    eng = Engine(N, R, D, dev)
    P, G = FlatParams(N, R, D, dev), FlatParams(N, R, D, dev)
    P.load(reference_init(N, R, D, 89))
    opt = KerasAdam(P)
    adj = eng.adjacency(adj_mats)
    ed = eng.edges(tri, lab)
    allreduce = GradAllReduce(G.flat) if world > 1 else None
    del pos, neg, tri, lab

    def step():
        return eng.train_step(P, G, opt, adj, ed, t_global=T, allreduce=allreduce)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    eng.probe = {}
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    probe, eng.probe = eng.probe, None
    loss_val = float(loss.item()) / T

    # dominant kernel: largest total event time inside the timed steps
    T_local = ed.T
    flops_per_launch = {"tail_fwd_gemm": 2.0 * D * D * T_local, "tail_bwd_gemm": 2.0 * D * D * T_local,
                        "tail_dS_tn": 2.0 * D * D * T_local}
    kt = {k: [a.elapsed_time(b) for a, b in v] for k, v in probe.items()}
    dom = max(kt, key=lambda k: sum(kt[k]))
    avg_ms = statistics.mean(kt[dom])
    achieved = flops_per_launch[dom] / (avg_ms * 1e-3) / 1e12

    ms = elapsed / args.steps * 1e3
    result = {
        "metric": "adjacency edges/s per IDDGCN training step (pos fwd + neg fwd + bwd + Adam)",
        "value": M / (elapsed / args.steps),
        "unit": "edges/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": ms,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (seeded mutation-drug graph, reference-distribution random init)",
        "config": {"workload": cfg["name"], "num_nodes": N, "num_relations": R, "adjacency_edges": M,
                   "scored_edges": T, "scored_edges_per_gpu": T_local, "feat_dim": D,
                   "parallelism": f"edge-dp{world}"},
        "scored_edges_per_s": T / (elapsed / args.steps),
        "loss": loss_val,
        "kernel_ms_per_step": {k: sum(v) / args.steps for k, v in kt.items()},
        "roofline": {"kernel": dom, "bound": "mfma", "achieved": achieved, "peak": MFMA_F32_PEAK_TFLOPS,
                     "unit": "TFLOP/s", "frac": achieved / MFMA_F32_PEAK_TFLOPS, "traffic": None,
                     "avg_launch_ms": avg_ms, "flops_per_launch": flops_per_launch[dom]},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(cfg)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
