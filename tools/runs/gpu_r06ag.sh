#!/bin/bash
# round 6, pass ag: the layer-1 run combine with nontemporal row stores vs HEAD (tools/bench_mem.py, config-3 shape).
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06ag}
mkdir -p $OUT
timeout -k 10 400 python3 -u tools/bench_mem.py tools/runs/dbg/prev.so tools/runs/dbg/rcnt.so tools/runs/dbg/prev.so tools/runs/dbg/rcnt.so > "$OUT/ab_combine_nt.txt" 2>&1
rc=$?
echo "rc=$rc"
exit $rc
