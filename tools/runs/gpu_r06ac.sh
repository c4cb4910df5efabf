#!/bin/bash
# round 6, pass ac: the split E collectives test alone, with progress lines (the previous pass went silent in it).
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06ac}
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest "tests/test_gpu_parallel.py::test_node_sharded_split_e_collectives" -m gpu -x -v -s --timeout 150 --timeout-method thread 2>&1 | tee "$OUT/gpu_tests_split.txt"
rc=$?
echo "rc=$rc"
exit $rc
