#!/bin/bash
# round 5: fold-4 training records (data consistency table, summation-order sensitivity, epoch sweep)
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r05o
timeout -k 10 300 python -u tools/fold_data_consistency.py --train 0,4 --out gpurun_out/r05o/fold_data_consistency.json > gpurun_out/r05o/fold_data_consistency.log 2>&1 &&
timeout -k 10 600 python -u tools/fold_order_sensitivity.py --folds 0,4 --out gpurun_out/r05o/fold_order_sensitivity.json > gpurun_out/r05o/fold_order_sensitivity.log 2>&1 &&
timeout -k 10 300 python -u tools/fold_epoch_sweep.py --folds 4,0 --epochs 8000 --every 250 --out gpurun_out/r05o/fold_epoch_sweep.json > gpurun_out/r05o/fold_epoch_sweep.log 2>&1
