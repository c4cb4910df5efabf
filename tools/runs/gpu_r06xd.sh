#!/bin/bash
# round 6, pass xd: measurement records at the final HEAD (DistMult nontemporal stores) — rocprofv3 kernel traces and the two PMC passes (FETCH_SIZE, WRITE_SIZE;
# separate runs, MI355X_MICROARCH.md §HBM) of the bench command of configs 3, 4 and 5, for profiles/r06 (kernel
# stats, per-kernel traffic, whole-step HBM bytes against engine.step_bytes_impl).
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06xd}
mkdir -p $OUT
B3="bench.py --no-cpu-baseline --no-other-mode --no-fold0-auc --also none --steps 5 --warmup 2"
B4="bench.py --config 4 --no-cpu-baseline --no-other-mode --no-fold0-auc --also none --steps 2 --warmup 1"
B5="bench.py --config 5 --no-cpu-baseline --no-other-mode --no-fold0-auc --also none --steps 2 --warmup 1"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/c3_trace" -o run --output-format csv -- python3 $B3 > "$OUT/c3_traced.log" 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d "$OUT/c3_fetch" -o run --output-format csv -- python3 $B3 > "$OUT/c3_fetch.log" 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d "$OUT/c3_write" -o run --output-format csv -- python3 $B3 > "$OUT/c3_write.log" 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/c5_trace" -o run --output-format csv -- python3 $B5 > "$OUT/c5_traced.log" 2>&1 &&
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/c5_fetch" -o run --output-format csv -- python3 $B5 > "$OUT/c5_fetch.log" 2>&1 &&
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/c5_write" -o run --output-format csv -- python3 $B5 > "$OUT/c5_write.log" 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/c4_trace" -o run --output-format csv -- python3 $B4 > "$OUT/c4_traced.log" 2>&1 &&
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/c4_fetch" -o run --output-format csv -- python3 $B4 > "$OUT/c4_fetch.log" 2>&1 &&
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/c4_write" -o run --output-format csv -- python3 $B4 > "$OUT/c4_write.log" 2>&1
rc=$?
echo "rc=$rc"
exit $rc
