"""TensorFlow 2.7's random initialisers, replayed on the host (the reference's weight init, IDDGCN.py:25-58,
92-101, 221-224, under the global seed of IDDGCN.py:292).

TensorFlow is not importable here, so its published algorithm is restated (third-party semantics of
tensorflow==2.7.0 / keras==2.7.0, README.md:17-19):

  * ``tf.random.set_seed(s)`` keeps a Python ``random.Random(s)`` in the eager context; an op without an op
    seed takes ``rng.randint(0, 2**31 - 1)`` (context.internal_operation_seed), an op with one takes it as
    given; the op's attributes are (seed, seed2) = (s % (2**31 - 1), op_seed % (2**31 - 1))
    (random_seed.get_seed).
  * Keras 2.7's initialisers: RandomUniform / RandomNormal / glorot_uniform call the STATEFUL
    ``tf.random.uniform`` / ``tf.random.normal`` with ``seed=`` the initialiser's seed (None when unseeded);
    'uniform' is RandomUniform(-0.05, 0.05), glorot_uniform is uniform in +-sqrt(6 / (fan_in + fan_out)).
  * The CPU kernels (random_op.cc, philox_random.h, random_distributions.h): a PhiloxRandom(seed, seed2)
    generator — key (seed lo, seed hi), counter (0, 0, seed2 lo, seed2 hi) — Philox4x32-10, one call per 4
    outputs; uniform float = the 23 low bits as the mantissa of a float in [1, 2), minus 1; normal float =
    Box-Muller on the pair (u1 clipped at 1e-7, v1 = float(2 pi u2), sqrt(-2 log u1) x sincos(v1)).  Each
    execution reserves output_count x 256 counter steps, and eager mode caches one kernel per (op, seed, seed2),
    so a second call of the same seeded op continues 256 x n counter steps further on.
  * ``tf.random.uniform(minval, maxval)``: ``rnd * (maxval - minval) + minval`` in float32 unless both bounds are
    the Python ints 0 and 1; ``tf.random.normal``: ``rnd * stddev + mean``.

Pinned bit for bit by the reference's own files (tests/test_tf_random.py): the three layers' relation_weights
(never trained) of the bundled fold 0/1/2/4 weights are op seeds #0, #2, #4 of Random(89) and those of fold 3
#7, #9, #11 (a second model in its process); the entity-embedding rows of the entities no training triple
touches (gradient zero through 5000 Adam steps: folds 0, 1, 4) are the RandomUniform(0, 1, seed=89) stream from
counter 0.  The normal draws (relation / self kernels, DistMult's relation embedding) go through the host libm's
logf / sincosf like TF's CPU kernel; every one of them is trained in the bundled files, so their bits are
unpinned.
"""
import ctypes
import ctypes.util
import math
import random

import numpy as np

_M32 = np.uint64(0xFFFFFFFF)
_MAXINT32 = 2 ** 31 - 1
_MUL_A, _MUL_B = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
_KEY_A, _KEY_B = 0x9E3779B9, 0xBB67AE85


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    """Philox4x32-10 (philox_random.h ComputeSingleRound / RaiseKey) on uint64 arrays holding uint32 values;
    returns the four output words."""
    c0, c1, c2, c3 = (np.asarray(c, dtype=np.uint64) for c in (c0, c1, c2, c3))
    k0, k1 = int(k0), int(k1)
    for r in range(10):
        p0 = _MUL_A * c0
        p1 = _MUL_B * c2
        hi0, lo0 = p0 >> np.uint64(32), p0 & _M32
        hi1, lo1 = p1 >> np.uint64(32), p1 & _M32
        c0, c1, c2, c3 = hi1 ^ c1 ^ np.uint64(k0), lo1, hi0 ^ c3 ^ np.uint64(k1), lo0
        if r < 9:
            k0, k1 = (k0 + _KEY_A) & 0xFFFFFFFF, (k1 + _KEY_B) & 0xFFFFFFFF
    return c0, c1, c2, c3


def philox_words(seed, seed2, base, n_calls, chunk=1 << 20):
    """The uint32 words of ``n_calls`` generator calls starting ``base`` steps into the stream of
    PhiloxRandom(seed, seed2), in output order (4 per call)."""
    out = np.empty(4 * n_calls, dtype=np.uint32)
    k0, k1 = seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF
    for a in range(0, n_calls, chunk):
        b = min(n_calls, a + chunk)
        g = np.arange(base + a, base + b, dtype=np.uint64)          # 128-bit counter = (g, seed2)
        r = philox4x32_10(g & _M32, g >> np.uint64(32), np.uint64(seed2 & 0xFFFFFFFF),
                          np.uint64((seed2 >> 32) & 0xFFFFFFFF), k0, k1)
        out[4 * a:4 * b] = np.stack(r, axis=1).astype(np.uint32).ravel()
    return out


def uint32_to_float(x):
    """random_distributions.h Uint32ToFloat: [0, 1) from the 23 low bits."""
    return (((np.asarray(x, dtype=np.uint32) & np.uint32(0x7FFFFF)) | np.uint32(127 << 23)).view(np.float32)
            - np.float32(1.0))


_libm = None


def _libm_fns():
    global _libm
    if _libm is None:
        lib = ctypes.CDLL(ctypes.util.find_library("m"))
        lib.logf.restype, lib.logf.argtypes = ctypes.c_float, [ctypes.c_float]
        lib.sincosf.restype = None
        lib.sincosf.argtypes = [ctypes.c_float, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_float)]
        _libm = lib
    return _libm


def box_muller(x0, x1):
    """random_distributions.h BoxMullerFloat on word pairs, through the host libm (as TF's CPU kernel)."""
    lib = _libm_fns()
    u1 = np.maximum(uint32_to_float(x0), np.float32(1.0e-7))
    v1 = (2.0 * math.pi * uint32_to_float(x1).astype(np.float64)).astype(np.float32)   # float(2 pi * u) in double
    lg = np.array([lib.logf(float(v)) for v in u1], dtype=np.float32)
    u2 = np.sqrt(np.float32(-2.0) * lg).astype(np.float32)
    s, c = ctypes.c_float(), ctypes.c_float()
    f0 = np.empty(len(v1), np.float32)
    f1 = np.empty(len(v1), np.float32)
    for i, v in enumerate(v1):
        lib.sincosf(float(v), ctypes.byref(s), ctypes.byref(c))
        f0[i], f1[i] = s.value, c.value
    return f0 * u2, f1 * u2


class TFRandom:
    """The eager random state after ``tf.random.set_seed(global_seed)`` in a fresh process: op-seed draws and the
    per-(op, seed, seed2) kernel cache."""

    def __init__(self, global_seed):
        self.global_seed = int(global_seed)
        self._rng = random.Random(self.global_seed)
        self._kernels = {}

    def get_seed(self, op_seed=None):
        """random_seed.get_seed in eager mode with a global seed set."""
        if op_seed is None:
            op_seed = self._rng.randint(0, _MAXINT32)
        seeds = (self.global_seed % _MAXINT32, int(op_seed) % _MAXINT32)
        return (0, _MAXINT32) if seeds == (0, 0) else seeds

    def _reserve(self, op, seed, n_out):
        """The kernel's stream position for this execution (ReserveRandomOutputs(n, 256))."""
        key = (op, seed)
        base = self._kernels.get(key, 0)
        self._kernels[key] = base + 256 * n_out
        return base

    def uniform(self, shape, minval=0, maxval=1, seed=None):
        """tf.random.uniform (float32)."""
        s = self.get_seed(seed)
        n = int(np.prod(shape))
        base = self._reserve("RandomUniform", s, n)
        rnd = uint32_to_float(philox_words(s[0], s[1], base, (n + 3) // 4)[:n])
        if not (isinstance(minval, int) and minval == 0 and isinstance(maxval, int) and maxval == 1):
            lo, hi = np.float32(minval), np.float32(maxval)
            rnd = (rnd * (hi - lo)).astype(np.float32) + lo
        return rnd.astype(np.float32).reshape(shape)

    def normal(self, shape, mean=0.0, stddev=1.0, seed=None):
        """tf.random.normal (float32)."""
        s = self.get_seed(seed)
        n = int(np.prod(shape))
        base = self._reserve("RandomStandardNormal", s, n)
        w = philox_words(s[0], s[1], base, (n + 3) // 4)
        f0, f1 = box_muller(w[0::2], w[1::2])
        rnd = np.empty(len(w), np.float32)
        rnd[0::2], rnd[1::2] = f0, f1
        rnd = rnd[:n]
        rnd = (rnd * np.float32(stddev)).astype(np.float32) + np.float32(mean)
        return rnd.astype(np.float32).reshape(shape)

    def glorot_uniform(self, shape, seed=None):
        """keras VarianceScaling(1, 'fan_avg', 'uniform') on a 2-D shape."""
        fan_in, fan_out = shape[0], shape[1]
        limit = math.sqrt(3.0 * 1.0 / max(1.0, (fan_in + fan_out) / 2.0))
        return self.uniform(shape, -limit, limit, seed)


def draw_model(tf, num_entities, num_relations, dim, seed=89):
    """Every weight of one get_IDDGCN_Model(..., seed) (IDDGCN.py:201-285) drawn from the eager state ``tf`` in
    creation order: the entity embedding (built at its first call, :226), then per IDDGCN_Layer (weights created
    in __init__, :23-58) relation_kernels, self_kernel, relation_weights, W_alpha, b_alpha, then DistMult's
    rel_embedding (built at its call, :90-101).  Returns the engine's names (E, K1, S1, relw1, Wa1, ba1, ..., rel)."""
    N, R, D = num_entities, num_relations, dim
    p = {"E": tf.uniform((N, D), 0, 1, seed=seed)}
    for l in (1, 2, 3):
        p[f"K{l}"] = tf.normal((R, D, D), 0.0, 1.0, seed=seed)
        p[f"S{l}"] = tf.normal((D, D), 0.0, 1.0, seed=seed)
        p[f"relw{l}"] = tf.uniform((R,), -0.05, 0.05)
        p[f"Wa{l}"] = tf.glorot_uniform((D, R))
        p[f"ba{l}"] = np.zeros((R,), np.float32)
    p["rel"] = tf.normal((R, D), 0.0, 1.0, seed=seed)
    return p


def reference_init(num_entities, num_relations, dim, seed=89, models_before=0, extra_op_seeds=0):
    """The reference's initial weights for a model built after ``tf.random.set_seed(seed)`` (IDDGCN.py:292) in a
    fresh process, or as the (models_before + 1)-th model of its process with ``extra_op_seeds`` further unseeded
    ops drawn in between (the bundled fold-3 weights: models_before=1, extra_op_seeds=1 — their relation_weights
    are op seeds #7, #9, #11)."""
    tf = TFRandom(seed)
    for _ in range(models_before):
        draw_model(tf, num_entities, num_relations, dim, seed)
    for _ in range(extra_op_seeds):
        tf.get_seed()
    return draw_model(tf, num_entities, num_relations, dim, seed)
