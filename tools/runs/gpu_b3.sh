#!/bin/bash
# bf16x3 GEMM mode on the box: smoke, the model-level GPU tests that run it, and a config-3 bench line in
# that mode (exact timed beside it as other_gemm_mode).  Every GPU step has its own time limit; a crash, hang
# or fault stops the script (pytest rc 1 = test failures only: the next steps still run).
# usage (repo root, on the box): bash tools/gpu_b3.sh <tag> [pytest -k expression]
set -o pipefail
TAG=${1:-b3}; K=${2:-"bf16x3 or deterministic or reentrant"}
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?
tail -6 $OUT/smoke.log; [ $rc -ne 0 ] && { echo "smoke rc=$rc"; exit $rc; }
timeout -k 10 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests -m gpu -k "$K" > $OUT/tests.log 2>&1; rc=$?
tail -4 $OUT/tests.log; [ $rc -gt 1 ] && { echo "pytest rc=$rc"; exit $rc; }
timeout -k 10 300 python -u bench.py --gemm bf16x3 --steps 10 --warmup 3 --also none --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err; rc=$?
tail -c 1500 $OUT/bench.json; [ $rc -ne 0 ] && { tail -5 $OUT/bench.err; exit $rc; }
echo done
