#!/bin/bash
# round 6, pass v: in-kernel clock of the row GEMM, HEAD form vs late gathers two tiles ahead (fine stamps of tiles
# 402-414 plus s_memrealtime), alternated twice.
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06v}
mkdir -p $OUT
for k in 1 2; do
  timeout -k 10 200 python3 -u tools/runs/dbg/stamp_fwd_fine.py tools/runs/dbg/stamp_l2_mid.so --case fwd_combine > "$OUT/clock_2ahead_$k.txt" 2>&1 &&
  timeout -k 10 200 python3 -u tools/runs/dbg/stamp_fwd_fine.py tools/runs/dbg/stamp_fine_mid.so --case fwd_combine > "$OUT/clock_head_$k.txt" 2>&1 || exit $?
done
echo "rc=0"
