#!/bin/bash
# Node-row partitioning evidence and configs 4/5 kernel profiles at HEAD.  usage (repo root, on the box):
#   bash tools/gpu_scale.sh <tag>
# 1. tools/node_shard_dryrun.py: every rank's compute of an 8-way node-row partitioned step, timed on this GPU
#    (configs 3, 4, 5), beside the single-GPU step;
# 2. rocprofv3 --kernel-trace --stats of the config-4 and config-5 bench (3 timed steps, 1 warm-up).
set -o pipefail
OUT=gpurun_out/${1:-scale}
mkdir -p "$OUT"
export TMPDIR=/tmp
for c in 3 4 5; do
  timeout -k 10 300 python -u tools/node_shard_dryrun.py $c 8 3 > "$OUT/dryrun_cfg$c.jsonl" 2>&1 || { echo "dryrun $c failed"; tail "$OUT/dryrun_cfg$c.jsonl"; exit 3; }
  tail -1 "$OUT/dryrun_cfg$c.jsonl" | cut -c1-400
done
for c in 4 5; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace_cfg$c" -o run --output-format csv -- python3 bench.py --config $c --also none --no-cpu-baseline --no-other-mode --steps 3 --warmup 1 > "$OUT/bench_cfg$c.log" 2>&1 || { echo "prof $c failed"; tail "$OUT/bench_cfg$c.log"; exit 3; }
  tail -c 400 "$OUT/bench_cfg$c.log"; echo
done
echo done
