#!/bin/bash
# round 5: 8-way node-row partition dry runs at HEAD (configs 5 and 4)
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r05d2
timeout -k 10 500 python -u tools/node_shard_dryrun.py 5 8 3 all > gpurun_out/r05d2/dryrun_cfg5.jsonl 2>&1 &&
timeout -k 10 500 python -u tools/node_shard_dryrun.py 4 8 3 all > gpurun_out/r05d2/dryrun_cfg4.jsonl 2>&1
