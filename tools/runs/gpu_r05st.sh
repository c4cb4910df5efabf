#!/bin/bash
# round 5: fused sigma' backward + dS TN (ABI 11) — kernel tests, config-5 tests, A/B on config-5 buffers
set -o pipefail
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r05st
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_bf16.py -k "sigma_tn" > $OUT/tests_kernel.txt 2>&1 &&
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bf16.py tests/test_gpu_config5.py tests/test_gpu_reentrant.py > $OUT/tests.txt 2>&1 &&
timeout -k 10 400 python -u tools/ab_sigma_tn.py 5 > $OUT/ab.txt 2>&1
