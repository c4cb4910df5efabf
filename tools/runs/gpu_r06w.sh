#!/bin/bash
# round 6, pass w: per-workgroup wall time of the layer-3 forward row GEMM in a real config-3 step (load balance).
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06w}
mkdir -p $OUT
timeout -k 10 300 python3 -u tools/runs/dbg/wg_times.py tools/runs/dbg/wgt.so > "$OUT/wg_times.txt" 2>&1
rc=$?
echo "rc=$rc"
exit $rc
