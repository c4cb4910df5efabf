"""Re-entrancy of the C-ABI ("re-entrant across streams and devices"; include/iddgcn.h ABI 6).

The GEMM operand precision is an argument of every GEMM call, not process state: two engines in different
modes (exact f32 and split-fp16 operands) running at the same time — each on its own HIP stream, issued from
its own host thread, so their launches interleave on the host and their kernels overlap on the device —
each give bitwise the results of the same engine run alone.

The same holds inside one engine: ``Engine.overlap`` runs the layer-2/3 tail reductions of the backward on a side
stream beside the dS TN and the sigma' GEMM (engine.Engine.backward); four training steps with it are bitwise the
steps without it, eagerly and through the HIP-graph replay (engine.GraphedTrainStep captures the fork / join).
"""
import threading

import numpy as np
import pytest
import torch

from iddgcn_amd.engine import Engine, FlatParams, GraphedTrainStep, KerasAdam
from iddgcn_amd.graph import get_adj_mats
from iddgcn_amd.utils import synthetic_graph

pytestmark = pytest.mark.gpu


def _params(N, R, D, seed):
    rng = np.random.default_rng(seed)
    p = {"E": rng.standard_normal((N, D)) / np.sqrt(D)}
    for l in (1, 2, 3):
        p[f"K{l}"] = rng.standard_normal((R, D, D)) / D
        p[f"S{l}"] = rng.standard_normal((D, D)) / np.sqrt(D)
        p[f"Wa{l}"] = rng.standard_normal((D, R)) / np.sqrt(D)
        p[f"ba{l}"] = rng.standard_normal(R) * 0.1
    p["rel"] = rng.standard_normal((R, D))
    return {k: v.astype(np.float32) for k, v in p.items()}


def test_two_engines_two_modes_two_streams_bitwise(cuda):
    N, R, D = 4000, 2, 256
    pos, neg = synthetic_graph(N, R, 40_000, seed=13)
    tri = np.concatenate([pos, neg])
    lab = np.concatenate([np.ones(len(pos)), np.zeros(len(neg))])
    jobs = {}
    for mode in ("exact", "split", "bf16x3"):
        eng = Engine(N, R, D, cuda, gemm=mode)
        P, G = FlatParams(N, R, D, cuda), FlatParams(N, R, D, cuda)
        P.load(_params(N, R, D, 3))
        jobs[mode] = dict(eng=eng, P=P, G=G, adj=eng.adjacency(get_adj_mats(pos, N, R)), ed=eng.edges(tri, lab))

    def run(j, reps=1):
        out = None
        for _ in range(reps):
            loss, p, s = j["eng"].loss_and_grads(j["P"], j["G"], j["adj"], j["ed"], logits=True)
            out = (loss.clone(), p.clone(), s.clone(), j["G"].buf.clone())
        return out

    alone = {m: run(j) for m, j in jobs.items()}
    torch.cuda.synchronize()
    # the two modes really differ (otherwise the test below would prove nothing)
    assert not torch.equal(alone["exact"][3], alone["split"][3])
    assert not torch.equal(alone["exact"][3], alone["bf16x3"][3])

    results, errors = {}, []

    def worker(mode):
        try:
            st = torch.cuda.Stream(device=cuda)
            with torch.cuda.stream(st):
                results[mode] = run(jobs[mode], reps=3)
            st.synchronize()
        except Exception as e:        # reported below
            errors.append(repr(e))

    threads = [threading.Thread(target=worker, args=(m,)) for m in jobs]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=120)
    torch.cuda.synchronize()
    assert not errors, errors
    for mode in jobs:
        for a, b in zip(alone[mode], results[mode]):
            assert torch.equal(a, b), mode


@pytest.mark.parametrize("gemm,R,features", [("exact", 2, "f32"), ("bf16x3", 2, "f32"), ("split", 8, "bf16")])
def test_overlap_backward_bitwise_eager_and_graphed(gemm, R, features, cuda):
    """Engine.overlap: the layer-2/3 tail reductions on a side stream (fork after everything queued, join before the
    head side).  R = 8 with bf16 edge tables (config 5's mode) forks the fused tail + head-term reduction
    (tail_seg_reduce_head: dP, dWedge and the per-node <dO, P_r> into dwh, read by head_dz after the join): bitwise the
    single-stream step, eager and HIP-graph replayed."""
    N, D = 4000, 256
    pos, neg = synthetic_graph(N, R, 40_000, seed=17)
    tri = np.concatenate([pos, neg])
    lab = np.concatenate([np.ones(len(pos)), np.zeros(len(neg))])
    params = _params(N, R, D, 5)

    def four_steps(overlap, graphed):
        eng = Engine(N, R, D, cuda, gemm=gemm, features=features)
        eng.overlap = overlap
        P, G = FlatParams(N, R, D, cuda), FlatParams(N, R, D, cuda)
        P.load(params)
        opt = KerasAdam(P)
        adj, ed = eng.adjacency(get_adj_mats(pos, N, R)), eng.edges(tri, lab)
        eng.train_step(P, G, opt, adj, ed)              # eager first step (creates every workspace)
        if graphed:
            step = GraphedTrainStep(eng, P, G, opt, adj, ed, n_steps=3)
            for _ in range(3):
                step.replay()
        else:
            for _ in range(3):
                eng.train_step(P, G, opt, adj, ed)
        torch.cuda.synchronize()
        return P.buf.clone(), G.buf.clone()

    base = four_steps(False, False)
    for overlap, graphed in ((True, False), (True, True), (False, True)):
        got = four_steps(overlap, graphed)
        assert torch.equal(got[0], base[0]) and torch.equal(got[1], base[1]), (gemm, overlap, graphed)
