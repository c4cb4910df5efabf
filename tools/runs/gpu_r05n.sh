#!/bin/bash
# round 5: node-row E ownership tests (after the world-3 assertion fix), fold-4 init probe, dry runs with owner Adam
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r05n
timeout -k 10 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread "tests/test_gpu_parallel.py::test_node_sharded_owner_e_adam" "tests/test_gpu_parallel.py::test_overlapped_adam_equals_adam_after_allreduce" tests/test_gpu_rccl.py > gpurun_out/r05n/tests.txt 2>&1 &&
timeout -k 10 300 python -u tools/fold4_init_probe.py --m 0,1,2,3,4 --out gpurun_out/r05n/fold4_init.json > gpurun_out/r05n/fold4_init.log 2>&1 &&
timeout -k 10 400 python -u tools/node_shard_dryrun.py 4 8 3 all > gpurun_out/r05n/dryrun_cfg4.jsonl 2>&1 &&
timeout -k 10 400 python -u tools/node_shard_dryrun.py 5 8 3 all > gpurun_out/r05n/dryrun_cfg5.jsonl 2>&1
