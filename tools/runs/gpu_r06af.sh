#!/bin/bash
# round 6, pass af: DistMult (distmult_heads_kernel) with a 5 / 6 waves-per-SIMD occupancy target vs HEAD (4),
# tools/bench_tailseg.py (DistMult at the config-3 and config-5 shapes, the tail reductions unchanged).
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06af}
mkdir -p $OUT
timeout -k 10 500 python3 -u tools/bench_tailseg.py tools/runs/dbg/prev.so tools/runs/dbg/dm5.so tools/runs/dbg/dm6.so tools/runs/dbg/prev.so > "$OUT/ab_dm_occupancy.txt" 2>&1
rc=$?
echo "rc=$rc"
exit $rc
