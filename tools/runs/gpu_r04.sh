#!/bin/bash
# Round-4 GPU pass.  usage (repo root, on the box): bash tools/gpu_r04.sh <tag> <what> [pytest args...]
#   what = tests  : the given pytest selection only
#          bench  : the selection, then smoke() and the default bench line
#          prof   : the selection, smoke, default bench, then rocprofv3 kernel-trace/stats and the two PMC passes
#                   (FETCH_SIZE, WRITE_SIZE: separate runs) of the headline bench command
# Test failures (pytest rc 1) do not stop the measurement steps; a crash, hang or fault (any other rc) does, and
# every GPU step has its own time limit.
set -o pipefail
TAG=$1; WHAT=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
export IDDGCN_PARITY_LOG=$PWD/$OUT/fullsize_grads.jsonl
rc=0
if [ $# -gt 0 ]; then
  timeout -k 10 1000 python -u -m pytest "$@" -m gpu -v -rf --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
  rc=$?
  grep -E "PASSED|FAILED|ERROR|passed|failed" "$OUT/gpu_tests.log" | tail -40
  if [ $rc -gt 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
fi
[ "$WHAT" = tests ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo "smoke failed"; tail "$OUT/smoke.log"; exit 3; }
tail -5 "$OUT/smoke.log"
timeout -k 10 600 python -u bench.py > "$OUT/bench_default.json.log" 2>&1 || { echo "bench failed"; tail -20 "$OUT/bench_default.json.log"; exit 3; }
tail -c 1500 "$OUT/bench_default.json.log"
[ "$WHAT" = bench ] && exit $rc
B="bench.py --no-cpu-baseline --no-other-mode --also none --steps 5 --warmup 2"
timeout -k 10 120 python -u $B > "$OUT/bench_profiled_cmd.json.log" 2>&1 &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 $B > "$OUT/bench_traced.log" 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run --output-format csv -- python3 $B > "$OUT/pmc_fetch.log" 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run --output-format csv -- python3 $B > "$OUT/pmc_write.log" 2>&1
prc=$?
echo "tests rc=$rc profile rc=$prc"
exit $(( rc > prc ? rc : prc ))
