#!/bin/bash
# round 5: store-stall ablations of the w4 GEMM; node-row E ownership tests (owner Adam, RCCL world 1)
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r05j
timeout -k 10 200 python -u tools/w4_ablate.py ab_so/w0.so ab_so/w6.so ab_so/w7.so ab_so/w8.so > gpurun_out/r05j/ablate.txt 2>&1 &&
timeout -k 10 400 python -u tools/fold_order_sensitivity.py --folds 0,3,4 --out gpurun_out/r05j/fold_perm.json > gpurun_out/r05j/fold_perm.log 2>&1 &&
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_rccl.py "tests/test_gpu_parallel.py::test_node_sharded_owner_e_adam" "tests/test_gpu_parallel.py::test_overlapped_adam_equals_adam_after_allreduce" "tests/test_gpu_parallel.py::test_node_sharded_step_equals_full_batch" > gpurun_out/r05j/tests.txt 2>&1
