"""Negative sampling on the GPU (csrc/sampling.hip) vs the reference's host recipe (numpy legacy
RandomState, utils1.py:646-655) at the config-3 and config-4 sizes; checks bit-equality and prints
the times as one JSON line.  usage: python tools/bench_sampling.py
"""
import json
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from iddgcn_amd import ops  # noqa: E402
from oracle.ref_utils import generate_negative_samples_np  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    out = {}
    for M, N in ((2_000_000, 100_000), (20_000_000, 1_000_000)):
        rng = np.random.default_rng(0)
        tri = np.stack([rng.integers(0, N, M), rng.integers(0, 2, M), rng.integers(0, N, M)], 1)
        t0 = time.perf_counter()
        rh, _, rt = generate_negative_samples_np(tri[:, 0], tri[:, 1], tri[:, 2], N, 89)
        host_s = time.perf_counter() - t0
        tg = torch.as_tensor(tri, device=dev)
        ops.negative_samples(tg, N, 89)               # warm-up (module load, allocator)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        neg = ops.negative_samples(tg, N, 89)
        torch.cuda.synchronize()
        dev_s = time.perf_counter() - t0
        got = neg.cpu().numpy()
        out[f"M={M},N={N}"] = {"host_numpy_s": host_s, "device_s": dev_s, "speedup": host_s / dev_s,
                               "bit_equal": bool(np.array_equal(got[:, 0], rh) and np.array_equal(got[:, 2], rt))}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
