#!/bin/bash
# round 6, pass yf: final validation at HEAD (after the split-E cache-key fix) — smoke, the whole GPU suite, the default bench line, and a two-rank
# node-row bench over gloo on the one GPU (a rehearsal of the driver's multi-GPU line's code path).
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06yf}
mkdir -p $OUT
timeout -k 10 180 python3 -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 &&
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/gpu_tests.txt" 2>&1 &&
timeout -k 10 500 python3 -u bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" &&
IDDGCN_DIST_BACKEND=gloo timeout -k 10 600 python3 -u bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline --no-other-mode --no-fold0-auc --also none > "$OUT/bench_gloo2.json" 2> "$OUT/bench_gloo2.err"
rc=$?
echo "rc=$rc"
exit $rc
