#!/bin/bash
# round 5: node-level head chain split (R > 2) — tests touching it, the config-5 bench and kernel trace
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/r05w
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_bf16.py tests/test_gpu_config5.py tests/test_gpu_model.py tests/test_gpu_parallel.py > $OUT/tests.txt 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/c5_trace" -o run --output-format csv -- python3 bench.py --config 5 --also none --no-cpu-baseline --no-fold0-auc --steps 3 --warmup 1 > "$OUT/c5_traced.log" 2>&1
