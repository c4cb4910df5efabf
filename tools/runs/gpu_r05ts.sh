#!/bin/bash
# round 5: tail segmented reduction at R <= 2 with the next edge group loaded while this one is summed — A/B on the
# config-3 / config-5 shapes (base = HEAD source, pipe = -DTS_PIPE=1), outputs compared bitwise
set -o pipefail
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r05ts
mkdir -p $OUT
timeout -k 10 300 python -u tools/bench_tailseg.py varx/base.so varx/pipe.so varx/base.so varx/pipe.so > $OUT/ab.txt 2>&1
