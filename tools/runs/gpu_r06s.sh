#!/bin/bash
# round 6, pass s: fused sigma' + TN staging splits: 1 (waves 0-3 all, HEAD), 3 (0-3 dO rows, 4-7 X pairs),
# 4 (0-3 dO rows + own X, 4-7 own X); fused-kernel tests on the tree build.
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06s}
mkdir -p $OUT
timeout -k 10 500 python3 -u tools/ab_sigma_tn.py 5 --config 3 iddgcn_amd/libiddgcn_hip.so tools/runs/dbg/split3.so tools/runs/dbg/split4.so tools/runs/dbg/prev.so > "$OUT/ab_split.txt" 2>&1 &&
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_sigma_tn_b3.py -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/gpu_tests_st3.txt" 2>&1
rc=$?
echo "rc=$rc"
exit $rc
