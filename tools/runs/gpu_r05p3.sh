#!/bin/bash
# round 5: node-row partition with the fused sigma' + TN pass — parallel + RCCL tests, the 8-way config-5 dry run; and
# the fused kernel with both TN k-steps' fragments read before one wait (tnup) against HEAD (base)
set -o pipefail
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r05p3
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 500 --timeout-method thread tests/test_gpu_parallel.py tests/test_gpu_rccl.py > $OUT/tests_parallel.txt 2>&1 &&
timeout -k 10 500 python -u tools/node_shard_dryrun.py 5 8 3 all > $OUT/dryrun_cfg5.jsonl 2>&1 &&
timeout -k 10 500 python -u tools/ab_sigma_tn.py 5 varx/base.so varx/tnup.so > $OUT/ab_tnup.txt 2>&1
