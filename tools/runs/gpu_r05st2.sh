#!/bin/bash
# round 5: fused sigma' + TN, three buffers (stn3) vs four buffers with the waves staggered (stn4), config-5 buffers
set -o pipefail
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r05st2
mkdir -p $OUT
timeout -k 10 500 python -u tools/ab_sigma_tn.py 5 varx/stn3.so varx/stn4.so > $OUT/ab.txt 2>&1
