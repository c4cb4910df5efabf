#!/bin/bash
# round 5: R = 8 tail reduction with the chunk rows software-pipelined — bf16 tests, A/B on the config-5 buffers
# (cur = before), outputs compared bitwise
set -o pipefail
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r05v
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_bf16.py > $OUT/tests_bf16.txt 2>&1 &&
IDDGCN_CFG5_CASES="tail_seg R8 bf16,tail_seg R8 bf16 +dsum,tail+head fused" timeout -k 10 400 python -u tools/bench_cfg5_kernels.py varx/cur.so iddgcn_amd/libiddgcn_hip.so varx/cur.so iddgcn_amd/libiddgcn_hip.so > $OUT/ab.txt 2>&1
