#!/bin/bash
# One GPU-box pass: GPU tests, the default bench line, a rocprofv3 kernel-trace/stats run of the same
# bench command, and two PMC passes (FETCH_SIZE, WRITE_SIZE) for roofline.traffic.
# Every GPU step has its own time limit and the steps are chained with && (stop at the first failure).
# usage (from the repo root, on the box): bash tools/gpu_round.sh <tag> [pytest-args]
set -o pipefail
TAG=${1:-run}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
BENCH="bench.py --no-cpu-baseline --no-other-mode --no-fold0-auc --also none --steps 5 --warmup 2"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${2:-} > "$OUT/gpu_tests.log" 2>&1 &&
timeout -k 10 300 python -u bench.py > "$OUT/bench.json.log" 2>&1 &&
timeout -k 10 120 python -u $BENCH > "$OUT/bench_profiled_cmd.json.log" 2>&1 &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 $BENCH > "$OUT/bench_traced.log" 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run --output-format csv -- python3 $BENCH > "$OUT/pmc_fetch.log" 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run --output-format csv -- python3 $BENCH > "$OUT/pmc_write.log" 2>&1
rc=$?
echo "gpu_round rc=$rc"
exit $rc
