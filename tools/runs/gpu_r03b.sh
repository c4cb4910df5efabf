#!/bin/bash
# Round-3 GPU pass (bf16x3 headline): GPU tests (all failures listed), smoke, the default bench line, a
# rocprofv3 kernel-trace/stats run and two PMC passes (FETCH_SIZE, WRITE_SIZE: separate runs) of the headline
# bench command, and the parity report.  Test failures (pytest rc 1) do not stop the measurement steps; a
# crash, hang or fault (any other rc) does, and every GPU step has its own time limit.
# usage (repo root, on the box): bash tools/gpu_r03b.sh <tag> [pytest selection]
set -o pipefail
TAG=${1:-r03b}
SEL=${2:-tests}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest $SEL -m gpu -q -rf --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
rc=$?
tail -15 "$OUT/gpu_tests.log"
if [ $rc -gt 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo "smoke failed"; tail "$OUT/smoke.log"; exit 3; }
tail -5 "$OUT/smoke.log"
timeout -k 10 400 python -u bench.py > "$OUT/bench_default.json.log" 2>&1 || { echo "bench failed"; tail -20 "$OUT/bench_default.json.log"; exit 3; }
tail -c 3000 "$OUT/bench_default.json.log"
B="bench.py --no-cpu-baseline --no-other-mode --also none --steps 5 --warmup 2"  # default --gemm bf16x3
timeout -k 10 120 python -u $B > "$OUT/bench_profiled_cmd.json.log" 2>&1 &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 $B > "$OUT/bench_traced.log" 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run --output-format csv -- python3 $B > "$OUT/pmc_fetch.log" 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run --output-format csv -- python3 $B > "$OUT/pmc_write.log" 2>&1 &&
timeout -k 10 400 python -u tools/parity_report.py > "$OUT/parity_report.json" 2> "$OUT/parity.err"
prc=$?
echo "tests rc=$rc profile/parity rc=$prc"
exit $(( rc > prc ? rc : prc ))
