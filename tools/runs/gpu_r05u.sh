#!/bin/bash
# round 5: DistMult heads kernel with the per-edge scalar chain lane-parallel (one chain per group of U edges) — tests,
# A/B on the config-5 buffers (base = before), and a config-3 bench
set -o pipefail
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r05u
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bf16.py tests/test_gpu_kernels.py tests/test_gpu_model.py > $OUT/tests.txt 2>&1 &&
IDDGCN_CFG5_CASES="distmult_heads" timeout -k 10 400 python -u tools/bench_cfg5_kernels.py varx/base.so iddgcn_amd/libiddgcn_hip.so varx/base.so iddgcn_amd/libiddgcn_hip.so > $OUT/ab.txt 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --also none --no-cpu-baseline --no-fold0-auc > $OUT/bench_cfg3.json.log 2>&1
