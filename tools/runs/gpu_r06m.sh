#!/bin/bash
# round 6, pass m: phase stamps of the split-role fused sigma' + TN pass.
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06m}
mkdir -p $OUT
timeout -k 10 200 python3 -u tools/runs/dbg/stamp_sigma_tn.py tools/runs/dbg/stamp_st.so > "$OUT/stamp_sigma_tn_roles1.txt" 2>&1
rc=$?
echo "rc=$rc"
exit $rc
