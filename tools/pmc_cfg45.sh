#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes (one counter per rocprofv3 run) over short config-4 and config-5 bench runs,
# for roofline.traffic of the bench line's `also` entries.  usage: bash tools/pmc_cfg45.sh <tag>
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
for c in 4 5; do
  B="bench.py --config $c --also none --no-cpu-baseline --no-other-mode --steps 2 --warmup 1"
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/c${c}_fetch -o run --output-format csv -- python3 $B > $OUT/c${c}_fetch.log 2>&1 || exit $?
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/c${c}_write -o run --output-format csv -- python3 $B > $OUT/c${c}_write.log 2>&1 || exit $?
done
echo pmc_cfg45 done
