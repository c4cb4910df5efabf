#!/bin/bash
# From-scratch 5-fold training under both initialisation schemes (tools/train_folds.py), after the model /
# explainer / parallel GPU tests.  usage: bash tools/gpu_train.sh <tag> [seeds]
set -o pipefail
OUT=gpurun_out/$1
SEEDS=${2:-89,1,2,3,4}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -k "model or explain or parallel or h5" -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
tail -3 $OUT/tests.log
[ $rc -ne 0 ] && exit $rc
for init in tf27 independent; do
  timeout -k 10 500 python -u tools/train_folds.py --seeds $SEEDS --init $init --out $OUT/train_$init.json > $OUT/train_$init.log 2>&1 || exit $?
  tail -1 $OUT/train_$init.log
done
