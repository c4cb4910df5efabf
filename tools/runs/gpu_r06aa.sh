#!/bin/bash
# round 6, pass aa: batched bf16x3 node-level TN launches (one launch per layer instead of three) vs the previous
# build: the 3-entry call, whole config-3 steps; the TN kernel tests.
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06aa}
mkdir -p $OUT
timeout -k 10 200 python3 -u tools/ab_tn_batched.py iddgcn_amd/libiddgcn_hip.so tools/runs/dbg/prev.so > "$OUT/ab_tn_batched.txt" 2>&1 &&
timeout -k 10 400 python3 -u tools/ab_sigma_tn.py 3 --config 3 iddgcn_amd/libiddgcn_hip.so tools/runs/dbg/prev.so > "$OUT/ab_step.txt" 2>&1 &&
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_config3.py tests/test_gpu_model.py -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/gpu_tests_subset.txt" 2>&1
rc=$?
echo "rc=$rc"
exit $rc
