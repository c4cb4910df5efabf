#!/bin/bash
# round 5: split-mode TN (gemm_tn256_x3_kernel) without the __syncthreads fence drain after the conversion — tests,
# A/B at T = 4M (base = HEAD before, x3fix = after; outputs compared bitwise), config-5 bench line
set -o pipefail
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r05x3tn
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_config5.py > $OUT/tests.txt 2>&1 &&
timeout -k 10 300 python -u tools/ab_gemm.py --modes split --cases tn --rounds 3 varx/base.so varx/x3fix.so > $OUT/ab_tn.txt 2>&1 &&
timeout -k 10 400 python -u bench.py --config 5 --steps 3 --warmup 1 --also none --no-cpu-baseline --no-fold0-auc > $OUT/bench_cfg5.json.log 2>&1
