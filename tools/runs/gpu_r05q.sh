#!/bin/bash
# round 5: config-5 kernels A/B, weights hi + lo vs bf16 only (experiment build)
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r05q
IDDGCN_CFG5_CASES="sigma' bwd GEMM,fwd" timeout -k 10 600 python -u tools/bench_cfg5_kernels.py varx/base.so varx/w1.so varx/base.so varx/w1.so > gpurun_out/r05q/cfg5_w1_ab.txt 2>&1
