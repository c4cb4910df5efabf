#!/bin/bash
# round 5: the TN kernels' transposed reads in asm (no compiler vmcnt(0) drain before them) — TN tests, A/B of the
# bf16x3 TN at T = 4M (base = HEAD before, tnfix = after; outputs compared bitwise), config-3 bench
set -o pipefail
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r05tn
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_bf16.py tests/test_gpu_config3.py > $OUT/tests.txt 2>&1 &&
timeout -k 10 300 python -u tools/ab_gemm.py --modes bf16x3 --cases tn --rounds 3 varx/base.so varx/tnfix.so > $OUT/ab_tn.txt 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --also none --no-cpu-baseline --no-fold0-auc > $OUT/bench_cfg3.json.log 2>&1
