#!/bin/bash
# round 6, pass o: row GEMM fine stamps with the slab wait split by vmcnt (what the late wave waits for).
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06o}
mkdir -p $OUT
timeout -k 10 200 python3 -u tools/runs/dbg/stamp_fwd_fine.py tools/runs/dbg/stamp_fine.so --case fwd_combine > "$OUT/stamp_fwd_fine_split.txt" 2>&1
rc=$?
echo "rc=$rc"
exit $rc
