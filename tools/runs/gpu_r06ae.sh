#!/bin/bash
# round 6, pass ae: fused sigma' + TN staging split 5 (waves 0-3 stage + convert the dO rows at the top, waves 4-7 the
# X pairs after their sigma' MFMAs) vs HEAD (waves 0-3 everything).
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06ae}
mkdir -p $OUT
timeout -k 10 500 python3 -u tools/ab_sigma_tn.py 5 --config 3 iddgcn_amd/libiddgcn_hip.so tools/runs/dbg/split5.so > "$OUT/ab_split5.txt" 2>&1
rc=$?
echo "rc=$rc"
exit $rc
