#!/bin/bash
# One GPU-box correctness + speed pass: the GPU tests (every failure listed, not stopping at the first),
# then — only if pytest ended normally (rc 0 = green, rc 1 = test failures, no crash / hang / fault) —
# the default bench line and optional extra bench commands.
# usage (repo root, on the box): bash tools/gpu_check.sh <tag> [pytest selection] [-- extra bench args ...]
set -o pipefail
TAG=${1:-check}
SEL=${2:-tests}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest $SEL -m gpu -q -rf --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
rc=$?
tail -5 "$OUT/gpu_tests.log"
if [ $rc -gt 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 10 --warmup 3 > "$OUT/bench.log" 2>&1
brc=$?
tail -c 3000 "$OUT/bench.log"
echo "tests rc=$rc bench rc=$brc"
exit $(( rc > brc ? rc : brc ))
