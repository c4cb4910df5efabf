"""CPU oracle for the IDDGCN hot path — TEST INFRASTRUCTURE ONLY.

This package restates the reference algorithm (AhauBioinformatics/IDDGCN,
``prediction/IDDGCN.py`` and ``prediction/utils1.py``) on the CPU so that the
HIP implementation in ``iddgcn_amd`` can be checked against it.

Only ``tests/``, ``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of
``bench.py`` may import this package, and only as a checker / reported
baseline.  The product path (``iddgcn_amd``) never imports it and fails loudly
when its HIP library is missing.

Pinning status:
  * integer/graph path (fold splits, reverse triplets, sorted adjacency) is
    pinned bit-for-bit against the fold files bundled with the reference;
  * floating-point path is pinned end-to-end by the bundled trained weights
    (eval AUC per fold).  The reference ships no per-op output vectors, and
    TensorFlow 2.7 is not installable here, so op-level float parity with TF
    itself is unpinned; the oracle follows the op order of IDDGCN.py:60-109.
"""
