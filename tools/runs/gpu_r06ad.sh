#!/bin/bash
# round 6, pass ad: two-rank node-row bench over gloo on the one GPU with the split E collectives (--split-e) beside
# the default, both rank-consistent.
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06ad}
mkdir -p $OUT
IDDGCN_DIST_BACKEND=gloo timeout -k 10 500 python3 -u bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline --no-other-mode --no-fold0-auc --also none --split-e > "$OUT/bench_gloo2_split_e.json" 2> "$OUT/bench_gloo2_split_e.err"
rc=$?
echo "rc=$rc"
exit $rc
