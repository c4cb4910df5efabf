#!/bin/bash
# round 6, pass aj: whole config-3 steps, HEAD vs nontemporal DistMult do^3 stores only (ntd.so) vs every output
# store nontemporal (ntv.so), three alternated rounds; DistMult alone.
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06aj}
mkdir -p $OUT
timeout -k 10 300 python3 -u tools/ab_engine_flag.py --help > "$OUT/help.txt" 2>&1 || true
timeout -k 10 500 python3 -u tools/ab_sigma_tn.py 3 --config 3 tools/runs/dbg/prev.so tools/runs/dbg/ntd.so tools/runs/dbg/ntv.so > "$OUT/ab_step_nt.txt" 2>&1 &&
timeout -k 10 300 python3 -u tools/bench_tailseg.py tools/runs/dbg/prev.so tools/runs/dbg/ntd.so tools/runs/dbg/prev.so tools/runs/dbg/ntd.so > "$OUT/ab_dm_nt.txt" 2>&1
rc=$?
echo "rc=$rc"
exit $rc
