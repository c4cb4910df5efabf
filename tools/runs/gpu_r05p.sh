#!/bin/bash
# round 5: fold-4 records, part 2 (softmax-gauge distance for all folds; order sensitivity of folds 1-3)
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r05p
timeout -k 10 300 python -u tools/fold_gauge_distance.py --out gpurun_out/r05p/fold_gauge_distance.json > gpurun_out/r05p/fold_gauge_distance.log 2>&1 &&
timeout -k 10 600 python -u tools/fold_order_sensitivity.py --folds 1,2,3 --out gpurun_out/r05p/fold_order_sensitivity_123.json > gpurun_out/r05p/fold_order_sensitivity_123.log 2>&1
