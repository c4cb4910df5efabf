#!/bin/bash
# round 5: the layer-1 tail combine at R = 8 on MFMAs — bf16 tests, config-5 forward / step tests, A/B on the real
# config-5 buffers (cur = the VALU run combine)
set -o pipefail
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r05z2
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_bf16.py > $OUT/tests_bf16.txt 2>&1 &&
IDDGCN_CFG5_CASES="layer-1 tail combine" timeout -k 10 400 python -u tools/bench_cfg5_kernels.py varx/cur.so iddgcn_amd/libiddgcn_hip.so varx/cur.so iddgcn_amd/libiddgcn_hip.so > $OUT/ab.txt 2>&1 &&
timeout -k 10 600 python -u -m pytest -x -q --timeout 500 --timeout-method thread tests/test_gpu_config5.py > $OUT/tests_cfg5.txt 2>&1
