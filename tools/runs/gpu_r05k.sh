#!/bin/bash
# round 5: per-kernel tables of the config-5 8-way node-row partition — the single-GPU step and ranks 0 and 7
# (rocprofv3 kernel stats of tools/node_shard_dryrun.py), compared by tools/rank_kernel_table.py
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/r05k
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/full -o run --output-format csv -- python3 tools/node_shard_dryrun.py 5 8 3 none > $OUT/full.log 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/r0 -o run --output-format csv -- python3 tools/node_shard_dryrun.py 5 8 3 0 > $OUT/r0.log 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/r7 -o run --output-format csv -- python3 tools/node_shard_dryrun.py 5 8 3 7 > $OUT/r7.log 2>&1
for k in mfma lds mem valu; do
  timeout -k 10 200 tools/pkfma_probe 6 4096 $k > $OUT/pkfma_probe_$k.txt 2>&1 || exit 3
done
