#!/bin/bash
# round 6, pass d: the default bench line (configs 3 + 4 + 5, CPU baseline, fold-0 AUC), then a rocprofv3 kernel trace
# of the headline bench command (config 3) for the per-step kernel table.
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06d}
mkdir -p $OUT
BENCH="bench.py --no-cpu-baseline --no-other-mode --no-fold0-auc --also none --steps 5 --warmup 2"
timeout -k 10 400 python -u bench.py > $OUT/bench_default.json.log 2>&1 &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 $BENCH > "$OUT/bench_traced.log" 2>&1
rc=$?
echo "rc=$rc"
exit $rc
