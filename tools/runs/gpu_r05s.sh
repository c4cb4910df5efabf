#!/bin/bash
# round 5: config-5 logit error per bf16 edge-GEMM operand form; the bf16 tests
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r05s
timeout -k 10 300 python -u tools/cfg5_operand_error.py > gpurun_out/r05s/cfg5_operand_error.txt 2>&1 &&
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_bf16.py > gpurun_out/r05s/tests_bf16.txt 2>&1
