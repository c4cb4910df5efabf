#!/bin/bash
# round 6, pass q: config-5 fused sigma' + TN (bf16 tables) with split staging roles vs the previous build; bf16 tests.
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06q}
mkdir -p $OUT
timeout -k 10 600 python3 -u tools/ab_sigma_tn.py 5 --config 5 iddgcn_amd/libiddgcn_hip.so tools/runs/dbg/prev.so > "$OUT/ab_bf16_roles.txt" 2>&1 &&
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_bf16.py -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/gpu_tests_bf16.txt" 2>&1
rc=$?
echo "rc=$rc"
exit $rc
