#!/bin/bash
# Round-3 GPU pass: GPU tests (all failures listed), smoke, the default bench line (exact f32 headline),
# then a rocprofv3 kernel-trace/stats run of the headline bench command.  Test failures (pytest rc 1) do not
# stop the measurement steps; a crash, hang or fault (any other rc) does.
# usage (repo root, on the box): bash tools/gpu_r03.sh <tag> [pytest selection] [bench args ...]
set -o pipefail
TAG=${1:-r03}
SEL=${2:-tests}
shift 2 2>/dev/null
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest $SEL -m gpu -q -rf --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
rc=$?
tail -15 "$OUT/gpu_tests.log"
if [ $rc -gt 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
src=$?
tail -5 "$OUT/smoke.log"
if [ $src -ne 0 ]; then echo "smoke rc=$src: stopping"; exit $src; fi
BENCH="bench.py --no-cpu-baseline --also none --steps 10 --warmup 3 $*"
timeout -k 10 300 python -u $BENCH > "$OUT/bench.json.log" 2>&1 || { echo "bench failed"; tail -20 "$OUT/bench.json.log"; exit 3; }
tail -c 2500 "$OUT/bench.json.log"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 $BENCH --no-other-mode > "$OUT/bench_traced.log" 2>&1
prc=$?
echo "tests rc=$rc smoke rc=$src rocprof rc=$prc"
exit $(( rc > prc ? rc : prc ))
