#!/bin/bash
# round 6, pass r: bench lines of configs 3, 4, 5 after the row-GEMM prefetch removal and the split-role fused pass.
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06r}
mkdir -p $OUT
timeout -k 10 400 python3 -u bench.py --no-cpu-baseline --no-fold0-auc --also 4 5 > "$OUT/bench_all.json" 2> "$OUT/bench_all.err"
rc=$?
echo "rc=$rc"
exit $rc
