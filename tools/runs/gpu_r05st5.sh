#!/bin/bash
# round 5: fused sigma' + TN, TN MFMAs after the sigma-prime ones (il0) vs one per sigma-prime k-step (il1), config-5 buffers
set -o pipefail
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r05st5
mkdir -p $OUT
timeout -k 10 500 python -u tools/ab_sigma_tn.py 5 varx/il0.so varx/il1.so > $OUT/ab.txt 2>&1
