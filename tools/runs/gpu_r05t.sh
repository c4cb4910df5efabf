#!/bin/bash
# round 5: swizzled full-wave DMAs for the bf16 A rows (TN, R = 8 forward, v3 sigma' / forward) — the bf16 kernel
# tests, then A/B on the real config-5 buffers (base = before; libiddgcn_hip.so = after; tn4 = after for TN + fwd8 only,
# with four TN buffers)
set -o pipefail
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r05t
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_bf16.py > $OUT/tests_bf16.txt 2>&1 &&
IDDGCN_CFG5_CASES="TN bf16 (dS),sigma' bwd GEMM,sigma' bwd GEMM bf16 ops,fwd" timeout -k 10 500 python -u tools/bench_cfg5_kernels.py varx/base.so iddgcn_amd/libiddgcn_hip.so varx/tn4.so varx/base.so iddgcn_amd/libiddgcn_hip.so > $OUT/ab.txt 2>&1
