"""Negative sampling on the GPU (csrc/sampling.hip) vs the reference recipe restated on numpy
(oracle/ref_utils.generate_negative_samples_np = utils1.py:646-655): bit-exact, element for element,
over stream-block boundaries (624 words), single-entity and power-of-two-edge ranges (no rejection /
maximal rejection), seeds up to 2^32-1 and a config-3-sized draw."""
import numpy as np
import pytest
import torch

from iddgcn_amd import ops
from iddgcn_amd.sampling import generate_negative_samples_np, negative_samples
from oracle.ref_utils import generate_negative_samples_np as ref_negatives

pytestmark = pytest.mark.gpu


def test_mt19937_stream_matches_numpy(cuda):
    for seed in (0, 89, 2 ** 32 - 1):
        bg = np.random.MT19937()
        bg._legacy_seeding(seed)                       # np.random.seed(seed)
        ref = bg.random_raw(5000).astype(np.uint32)
        got = ops.mt19937_words(seed, 5000, cuda).cpu().numpy().view(np.uint32)
        assert np.array_equal(got, ref), seed


@pytest.mark.parametrize("M,N,seed", [(0, 845, 1), (1, 845, 7), (623, 845, 89), (624, 100_000, 0), (625, 2, 5),
                                      (100_003, 845, 123), (20_000, 1, 9), (50_000, 2 ** 20, 11),
                                      (50_000, 2 ** 20 + 1, 12), (300_000, 1_000_000, 2 ** 32 - 1),
                                      (2_000_000, 100_000, 89)])
def test_negative_samples_bit_exact(M, N, seed, cuda):
    rng = np.random.default_rng(M + N)
    h, r, t = rng.integers(0, N, M), rng.integers(0, 4, M), rng.integers(0, N, M)
    rh, rr, rt = ref_negatives(h, r, t, N, seed)
    gh, gr, gt = generate_negative_samples_np(h, r, t, N, seed, device=cuda)
    assert np.array_equal(gh, rh) and np.array_equal(gr, rr) and np.array_equal(gt, rt)


def test_negative_samples_gpu_tensor_in_out(cuda):
    tri = torch.randint(0, 845, (4000, 3), device=cuda)
    out = negative_samples(tri, 845, 3)
    assert out.is_cuda and out.shape == (4000, 3)
    a = tri.cpu().numpy()
    rh, _, rt = ref_negatives(a[:, 0], a[:, 1], a[:, 2], 845, 3)
    assert np.array_equal(out[:, 0].cpu().numpy(), rh) and np.array_equal(out[:, 2].cpu().numpy(), rt)
