#!/bin/bash
# round-5 final pass at HEAD: GPU tests, smoke, the default bench line, rocprofv3 kernel trace + the two PMC passes of
# the headline bench command (tools/gpu_round.sh), then kernel traces of configs 5 and 4.
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05x}
mkdir -p $OUT
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 &&
bash tools/gpu_round.sh ${TAG:-r05x} "-v --timeout 300" &&
for c in 5 4; do
  B="bench.py --config $c --also none --no-cpu-baseline --no-other-mode --no-fold0-auc --steps 2 --warmup 1"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/c${c}_trace" -o run --output-format csv -- python3 $B > "$OUT/c${c}_traced.log" 2>&1 || exit 3
done
