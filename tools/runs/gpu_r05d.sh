#!/bin/bash
# round 5: fold summation-order sensitivity, then the default bench at HEAD
set -o pipefail
mkdir -p gpurun_out/r05d
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u tools/fold_order_sensitivity.py --folds 0,1,2,3,4 --out gpurun_out/r05d/fold_order.json > gpurun_out/r05d/fold_order.log 2>&1 &&
timeout -k 10 400 python -u bench.py > gpurun_out/r05d/bench.log 2>&1
