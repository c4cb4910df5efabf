#!/bin/bash
# Round-4 measurement pass: rocprofv3 kernel-trace/stats and the two PMC passes (FETCH_SIZE, WRITE_SIZE: separate runs)
# of the config-3 headline bench command, then the same for configs 5 and 4 (bench --config N, 2-3 steps).  Every GPU
# step has its own time limit; the first failure stops the script.  usage (repo root, on the box):
#   bash tools/gpu_prof_r04.sh <tag>
set -o pipefail
OUT=gpurun_out/${1:-prof}
mkdir -p "$OUT"
export TMPDIR=/tmp
B="bench.py --no-cpu-baseline --no-other-mode --also none --steps 5 --warmup 2"
timeout -k 10 120 python -u $B > "$OUT/c3_bench.json.log" 2>&1 &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/c3_trace" -o run --output-format csv -- python3 $B > "$OUT/c3_traced.log" 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d "$OUT/c3_fetch" -o run --output-format csv -- python3 $B > "$OUT/c3_fetch.log" 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d "$OUT/c3_write" -o run --output-format csv -- python3 $B > "$OUT/c3_write.log" 2>&1 || { echo "config-3 profile failed"; exit 3; }
echo "config 3 done"
for c in 5 4; do
  B="bench.py --config $c --also none --no-cpu-baseline --no-other-mode --steps 2 --warmup 1"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/c${c}_trace" -o run --output-format csv -- python3 $B > "$OUT/c${c}_traced.log" 2>&1 &&
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/c${c}_fetch" -o run --output-format csv -- python3 $B > "$OUT/c${c}_fetch.log" 2>&1 &&
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/c${c}_write" -o run --output-format csv -- python3 $B > "$OUT/c${c}_write.log" 2>&1 || { echo "config-$c profile failed"; exit 3; }
  echo "config $c done"
done
