#!/bin/bash
# round 5: fused sigma' + TN, prefetch depth 2 / 3 / 4 tiles, config-5 buffers
set -o pipefail
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r05st4
mkdir -p $OUT
timeout -k 10 500 python -u tools/ab_sigma_tn.py 5 varx/pd2.so varx/pd3.so varx/pd4.so > $OUT/ab.txt 2>&1
