#!/bin/bash
# Config-5 pass: selected GPU tests (pytest -k expression), then a rocprofv3 kernel-trace/stats run of the
# config-5 bench (R = 8, bf16 features), then a config-3 bench line.  usage: bash tools/gpu_cfg5.sh <tag> "<-k expression>"
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -k "$2" -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
tail -3 $OUT/tests.log
[ $rc -gt 1 ] && exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --config 5 --also none --no-cpu-baseline --no-other-mode --steps 3 --warmup 1 > $OUT/bench.log 2>&1
brc=$?
[ $brc -ne 0 ] && { echo "bench rc=$brc"; exit $brc; }
timeout -k 10 200 python3 bench.py --also none --no-cpu-baseline --no-other-mode --steps 10 --warmup 3 > $OUT/bench3.log 2>&1
brc=$?
echo "tests rc=$rc bench rc=$brc"
exit $(( rc > brc ? rc : brc ))
