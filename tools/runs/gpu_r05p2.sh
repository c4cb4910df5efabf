#!/bin/bash
# round 5: node-row head-chain split (parallel tests + config-5 dry run), and the packed-fp32 op_sel probe
set -o pipefail
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r05p2
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 500 --timeout-method thread tests/test_gpu_parallel.py tests/test_gpu_rccl.py > $OUT/tests_parallel.txt 2>&1 &&
timeout -k 10 500 python -u tools/node_shard_dryrun.py 5 8 3 all > $OUT/dryrun_cfg5.jsonl 2>&1 &&
timeout -k 10 240 tools/pkfma_probe 20 4096 > $OUT/pkfma_probe.txt 2>&1
