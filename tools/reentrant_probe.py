"""Diagnose tests/test_gpu_reentrant.py: engines in different GEMM modes run alone, then concurrently (one
stream + host thread each); per mode, which outputs (loss, p, s, gradient tensors) differ and by how much.

usage: python tools/reentrant_probe.py mode1,mode2[,...] [reps]     (mode#k: another engine in that mode)
"""
import sys
import threading

import numpy as np
import torch

sys.path.insert(0, ".")
from iddgcn_amd.engine import Engine, FlatParams  # noqa: E402
from iddgcn_amd.graph import get_adj_mats  # noqa: E402
from iddgcn_amd.utils import synthetic_graph  # noqa: E402
from tests.test_gpu_reentrant import _params  # noqa: E402


WS = ["AE", "P", "X", "xt", "Wedge", "dWedge", "dP", "dAE", "dES", "dz", "dOn_a", "dOn_b"]


def main(modes, reps=3):
    cuda = torch.device("cuda", 0)
    N, R, D = 4000, 2, 256
    pos, neg = synthetic_graph(N, R, 40_000, seed=13)
    tri = np.concatenate([pos, neg])
    lab = np.concatenate([np.ones(len(pos)), np.zeros(len(neg))])
    jobs = {}
    for mode in modes:
        eng = Engine(N, R, D, cuda, gemm=mode.split("#")[0])        # "exact#2": a second engine, same mode
        P, G = FlatParams(N, R, D, cuda), FlatParams(N, R, D, cuda)
        P.load(_params(N, R, D, 3))
        jobs[mode] = dict(eng=eng, P=P, G=G, adj=eng.adjacency(get_adj_mats(pos, N, R)), ed=eng.edges(tri, lab))

    def run(j, n=1):
        outs = []
        for _ in range(n):
            loss, p, s = j["eng"].loss_and_grads(j["P"], j["G"], j["adj"], j["ed"], logits=True)
            ws = j["eng"].workspace(j["ed"].T, True)
            outs.append((loss.clone(), p.clone(), s.clone(), j["G"].buf.clone()) +
                        tuple(getattr(ws, k).clone() for k in WS))
        return outs

    alone = {m: run(j, 2) for m, j in jobs.items()}
    torch.cuda.synchronize()
    for m in modes:
        a, b = alone[m]
        print(m, "alone twice bitwise:", all(torch.equal(x, y) for x, y in zip(a, b)), flush=True)
    results = {}

    def worker(mode):
        st = torch.cuda.Stream(device=cuda)
        with torch.cuda.stream(st):
            results[mode] = run(jobs[mode], reps)
        st.synchronize()

    th = [threading.Thread(target=worker, args=(m,)) for m in modes]
    for t in th:
        t.start()
    for t in th:
        t.join()
    torch.cuda.synchronize()
    names = ["loss", "p", "s", "G"] + ["ws." + k for k in WS]
    for m in modes:
        G0 = jobs[m]["G"]
        for k, out in enumerate(results[m]):
            bad = []
            for nm, a, b in zip(names, alone[m][0], out):
                if not torch.equal(a, b):
                    d = (a.double() - b.double()).abs().max().item()
                    if nm == "G":       # which parameter tensors
                        off = 0
                        for name, view in G0.views.items():
                            n = view.numel()
                            if not torch.equal(a[off:off + n], b[off:off + n]):
                                bad.append(f"G.{name}:{(a[off:off + n] - b[off:off + n]).abs().max().item():.2e}")
                            off += n
                    else:
                        bad.append(f"{nm}:{d:.2e}")
            print(f"{m} concurrent rep {k}: {'bitwise' if not bad else ' '.join(bad)}", flush=True)


if __name__ == "__main__":
    main(sys.argv[1].split(","), int(sys.argv[2]) if len(sys.argv) > 2 else 3)
