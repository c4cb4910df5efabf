#!/bin/bash
# DistMult lane-parallel scalars + SQ counters of the R = 8 bf16 forward GEMM: GPU tests (-k selection), the
# config-3 bench line, then tools/pmc_gemm.sh on fwd8 and fwd.  usage: bash tools/gpu_dm.sh <tag> "<-k expr>"
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -k "$2" -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
tail -3 $OUT/tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python3 bench.py --also none --no-cpu-baseline --no-other-mode --steps 10 --warmup 3 > $OUT/bench3.log 2>&1 || exit $?
grep -h '"ms_per_step"' $OUT/bench3.log | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print('cfg3', d['ms_per_step'])"
bash tools/pmc_gemm.sh $OUT/pmc split fwd8 fwd
