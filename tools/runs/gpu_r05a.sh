#!/bin/bash
# round 5, first GPU pass: the new / changed tests, then smoke
set -o pipefail
mkdir -p gpurun_out/r05a
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_rccl.py tests/test_gpu_reentrant.py "tests/test_gpu_parallel.py::test_node_sharded_step_equals_full_batch" tests/test_gpu_config5.py > gpurun_out/r05a/tests.txt 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05a/smoke.log 2>&1
