#!/bin/bash
# round 5: HBM bytes per kernel of the config-5 step (FETCH_SIZE, WRITE_SIZE: one counter per rocprofv3 run)
set -o pipefail
OUT=gpurun_out/r05c5pmc
mkdir -p $OUT
export TMPDIR=/tmp
B="bench.py --config 5 --also none --no-cpu-baseline --no-other-mode --no-fold0-auc --steps 1 --warmup 1"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/c5_fetch -o run --output-format csv -- python3 $B > $OUT/c5_fetch.log 2>&1 &&
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/c5_write -o run --output-format csv -- python3 $B > $OUT/c5_write.log 2>&1
