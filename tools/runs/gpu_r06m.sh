#!/bin/bash
# round 6, pass m: phase stamps of the split-role fused sigma' + TN pass; fine stamps of the row GEMM loop.
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06m}
mkdir -p $OUT
timeout -k 10 200 python3 -u tools/runs/dbg/stamp_sigma_tn.py tools/runs/dbg/stamp_st.so > "$OUT/stamp_sigma_tn_roles1.txt" 2>&1 &&
timeout -k 10 200 python3 -u tools/runs/dbg/stamp_fwd_fine.py tools/runs/dbg/stamp_fine.so --case fwd_combine > "$OUT/stamp_fwd_fine.txt" 2>&1 &&
timeout -k 10 200 python3 -u tools/runs/dbg/stamp_fwd_fine.py tools/runs/dbg/stamp_fine.so --case bwd_dsig > "$OUT/stamp_bwd_fine.txt" 2>&1
rc=$?
echo "rc=$rc"
exit $rc
