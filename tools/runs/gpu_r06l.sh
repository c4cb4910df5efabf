#!/bin/bash
# round 6, pass l: fused sigma' + TN pass with split roles (waves 0-3 stage + convert for their SIMD, waves 4-7 only
# MFMAs + epilogue; ROLES 1 = conversions after the TN MFMAs, the tree) against ROLES 0 (round-6 form) and 2
# (conversions before the TN MFMAs): per launch and whole config-3 steps; then the fused-kernel tests.
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06l}
mkdir -p $OUT
timeout -k 10 400 python3 -u tools/ab_sigma_tn.py 5 --config 3 iddgcn_amd/libiddgcn_hip.so tools/runs/dbg/roles0.so tools/runs/dbg/roles2.so > "$OUT/ab_roles.txt" 2>&1 &&
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_sigma_tn_b3.py -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/gpu_tests_st3.txt" 2>&1
rc=$?
echo "rc=$rc"
exit $rc
