#!/bin/bash
# round 5: the bench line's fold-0 AUC field; a 2-rank gloo rehearsal of the multi-GPU bench (node rows, E owned by rows)
# with both ranks on the one GPU (configs 3, 4, 5)
set -o pipefail
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r05y
mkdir -p $OUT
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --also none --no-cpu-baseline --no-other-mode > $OUT/bench_fold0auc.json.log 2>&1 &&
IDDGCN_DIST_BACKEND=gloo timeout -k 10 800 python -u bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline --no-other-mode --also 4 5 > $OUT/bench_gloo2.json.log 2>&1
