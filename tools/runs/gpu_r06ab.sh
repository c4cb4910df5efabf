#!/bin/bash
# round 6, pass ab: the opt-in split E collectives — gloo world 2 / 3 node-row steps on one GPU against the unsplit
# collectives, the RCCL world-1 step bitwise, and the existing parallel tests.
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06ab}
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parallel.py tests/test_gpu_rccl.py -m gpu -x -v -s --timeout 400 --timeout-method thread > "$OUT/gpu_tests_parallel.txt" 2>&1
rc=$?
echo "rc=$rc"
exit $rc
