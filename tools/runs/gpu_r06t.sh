#!/bin/bash
# round 6, pass t: fine stamps of the row GEMM with the late waves' gathers two tiles ahead (why it measured slower),
# beside the HEAD form's fine stamps.
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06u}
mkdir -p $OUT
timeout -k 10 200 python3 -u tools/runs/dbg/stamp_fwd_fine.py tools/runs/dbg/stamp_l2_mid.so --case fwd_combine > "$OUT/stamp_fwd_fine_2ahead_mid.txt" 2>&1 &&
timeout -k 10 200 python3 -u tools/runs/dbg/stamp_fwd_fine.py tools/runs/dbg/stamp_fine_mid.so --case fwd_combine > "$OUT/stamp_fwd_fine_head_mid.txt" 2>&1
rc=$?
echo "rc=$rc"
exit $rc
