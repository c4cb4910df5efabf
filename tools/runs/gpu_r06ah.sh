#!/bin/bash
# round 6, pass ah: kernel / model / config-3 tests after the run combine's nontemporal stores.
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06ah}
mkdir -p $OUT
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_config3.py tests/test_gpu_bf16.py -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/gpu_tests_subset.txt" 2>&1
rc=$?
echo "rc=$rc"
exit $rc
