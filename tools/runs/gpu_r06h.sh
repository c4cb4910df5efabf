#!/bin/bash
# round 6, pass h: validation at HEAD — smoke, the whole GPU suite, the default bench line.
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06h}
mkdir -p $OUT
timeout -k 10 180 python3 -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 &&
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/gpu_tests.txt" 2>&1 &&
timeout -k 10 500 python3 -u bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.err"
rc=$?
echo "rc=$rc"
exit $rc
