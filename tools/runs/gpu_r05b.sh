#!/bin/bash
# round 5: the new / changed tests + smoke (product library = HEAD), then the bf16x3 GEMM A/B (ab_so/*.so)
set -o pipefail
mkdir -p gpurun_out/r05b
export PYTHONUNBUFFERED=1
timeout -k 10 240 python -u tools/ab_gemm.py --rounds 3 ab_so/base.so ab_so/regA.so > gpurun_out/r05b/ab_gemm.txt 2>&1 &&
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_rccl.py tests/test_gpu_reentrant.py "tests/test_gpu_parallel.py::test_node_sharded_step_equals_full_batch" tests/test_gpu_config5.py > gpurun_out/r05b/tests.txt 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05b/smoke.log 2>&1
