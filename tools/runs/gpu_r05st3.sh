#!/bin/bash
# round 5: HBM bytes of the fused sigma' + TN kernel on config-5 buffers (FETCH_SIZE, WRITE_SIZE passes)
set -o pipefail
OUT=gpurun_out/r05st3
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 tools/ab_sigma_tn.py -3 > $OUT/fetch.log 2>&1 &&
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 tools/ab_sigma_tn.py -3 > $OUT/write.log 2>&1
