#!/bin/bash
# round 6, pass e: the three layers' dK_r in one batched TN launch per relation (config 5's split node GEMMs): its
# test, config 5's and the R = 8 node-row tests, then the step A/B with Engine.merge_dk on and off at config 5.
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06e}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16.py -k "merged_dk or step_tracks" -x -v --timeout 200 --timeout-method thread > $OUT/tests_merge.txt 2>&1 &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_parallel.py -k "node_sharded_step and 8 or fused_tail_head" -x -v --timeout 300 --timeout-method thread > $OUT/tests_parallel.txt 2>&1 &&
timeout -k 10 600 python -u tools/ab_engine_flag.py --config 5 --flag merge_dk --reps 3 --rounds 3 > $OUT/ab_merge_dk_cfg5.txt 2>&1
rc=$?
echo "rc=$rc"
exit $rc
