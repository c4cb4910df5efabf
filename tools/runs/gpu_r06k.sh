#!/bin/bash
# round 6, pass k: s_memtime phase stamps of the fused sigma' + TN pass and of the row GEMM without its L2 prefetch.
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06k}
mkdir -p $OUT
timeout -k 10 200 python3 -u tools/runs/dbg/stamp_sigma_tn.py tools/runs/dbg/stamp_st.so > "$OUT/stamp_sigma_tn.txt" 2>&1 &&
timeout -k 10 200 python3 -u tools/runs/dbg/stamp_fwd.py tools/runs/dbg/stamp.so --case fwd_combine > "$OUT/stamp_fwd.txt" 2>&1 &&
timeout -k 10 200 python3 -u tools/runs/dbg/stamp_fwd.py tools/runs/dbg/stamp.so --case bwd_dsig > "$OUT/stamp_bwd.txt" 2>&1
rc=$?
echo "rc=$rc"
exit $rc
